#!/bin/bash
# r03: page-pinning threads for the host frontier -- the host-frontier and
# checkpoint GPU tests, then config 2 in auto mode with 4 (default) and 8
# pinning threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r03l}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_frontier.py tests/test_gpu_configs.py -k host > $O/pytest_hf.log 2>&1 || { echo "hf tests failed"; tail -30 $O/pytest_hf.log; exit 1; }
tail -2 $O/pytest_hf.log
export RMC_HOST_FRONTIER_GIB=245
t0=$(date +%s.%N); timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_pin4.txt 2>&1; echo "cfg2 pin4 rc=$? process wall $(python3 -c "import time; print(round(time.time() - $t0, 2))")"
grep -E "moved|host frontier:|depth 2[6-9]:" $O/ladder_Raft_n3v2e3_pin4.txt | cut -c1-200
t0=$(date +%s.%N); RMC_HF_PIN_THREADS=8 RMC_HF_PIN_AHEAD=64 timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_pin8.txt 2>&1; echo "cfg2 pin8 rc=$? process wall $(python3 -c "import time; print(round(time.time() - $t0, 2))")"
grep -E "moved|host frontier:|depth 2[6-9]:" $O/ladder_Raft_n3v2e3_pin8.txt | cut -c1-200
