#!/bin/bash
# A/B kernel timing: raft-tlaplus_amd/build (A) vs build_b (B), interleaved,
# each a full check of the bench cfg through the CLI (kernel ms from HIP events).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-Raft_n3v2e2}
for i in 1 2; do
  for v in ${BUILDS:-build build_b}; do
    timeout -k 10 120 ./raft-tlaplus_amd/$v/raftmc -deadlock -json -module Raft -config configs/$CFG.cfg > gpurun_out/ab_$v.txt 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_$v.txt; exit 1; }
    echo "$v $(tail -1 gpurun_out/ab_$v.txt)"
  done
done
