#!/bin/bash
# One gpurun call: smoke, GPU parity tests, Raft.cfg via the CLI.  Stops at the
# first step that dies (fault / abort / timeout) instead of running on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || [ "$rc" -eq 12 ]; }
timeout -k 10 180 python -u __graft_entry__.py > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft.cfg > gpurun_out/raft_cfg.txt 2>&1; rc=$?; echo "raftmc rc=$rc" | tee -a gpurun_out/raft_cfg.txt
exit 0
