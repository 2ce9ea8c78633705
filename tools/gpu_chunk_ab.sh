#!/bin/bash
# Chunk-size sweep on the bench cfg through the CLI.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ch in 1048576 2097152 4194304 1048576; do
  timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -chunk $ch -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/chunk_$ch.txt 2>&1 || { echo "chunk $ch failed"; tail -3 gpurun_out/chunk_$ch.txt; exit 1; }
  echo "chunk $ch $(tail -1 gpurun_out/chunk_$ch.txt)"
done
