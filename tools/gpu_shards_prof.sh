#!/bin/bash
# Kernel + copy time breakdown of the fingerprint-sharded protocol on one GPU:
# rocprofv3 --kernel-trace --memory-copy-trace --stats of one CLI check with W
# logical shards (SHARDS="1 8"), CFG (default Raft_n3v2e2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=${CFG:-Raft_n3v2e2}
for w in ${SHARDS:-1 8}; do
  timeout -k 10 ${LIMIT:-240} rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/shprof_$w -o run -- \
    ./raft-tlaplus_amd/build/raftmc -deadlock -json -shards $w -module Raft -config configs/$CFG.cfg > gpurun_out/shprof_$w.txt 2>&1; rc=$?
  echo "W=$w rc=$rc"; tail -1 gpurun_out/shprof_$w.txt
  [ $rc -eq 0 ] || exit $rc
done
find gpurun_out -name "*stats.csv" -path "*shprof*" | head -20
