#!/bin/bash
# One gpurun call: GPU parity tests, then N timed CLI checks of the bench cfg
# (kernel ms from librmc's HIP events).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-Raft_n3v2e2}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for i in 1 2 3; do
  timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config configs/$CFG.cfg > gpurun_out/ab.txt 2>&1 || { echo "raftmc failed"; tail -5 gpurun_out/ab.txt; exit 1; }
  tail -1 gpurun_out/ab.txt
done
