#!/bin/bash
# r03: the whole -m gpu suite with durations, then config 2 in the default
# (auto) host-frontier mode (early switch at a level boundary).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=30 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
grep -A32 "slowest" $O/pytest_gpu.log | head -34
export RMC_HOST_FRONTIER_GIB=245
timeout -k 10 600 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_auto.txt 2>&1; echo "cfg2 rc=$?"
grep -E "moved to host|windows|Error|states generated|depth of|Finished" $O/ladder_Raft_n3v2e3_auto.txt | cut -c1-200
