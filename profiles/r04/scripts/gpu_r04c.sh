#!/bin/bash
# r04: compact host-frontier rows.  The host-frontier / checkpoint / rung tests,
# then BASELINE config 2 with its levels on the host (245 GiB of pinned pages, as in r03),
# and the bench workload with the host frontier forced (PCIe-inclusive rate).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_frontier.py tests/test_gpu_checkpoint.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_hf.log 2>&1 || { echo "hf tests failed"; tail -30 $O/pytest_hf.log; exit 1; }
tail -2 $O/pytest_hf.log
export RMC_HOST_FRONTIER_GIB=245
timeout -k 10 420 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -hostfrontier 1 -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_hf1_compact.txt 2>&1; rc=$?
echo "cfg2 rc=$rc"; tail -4 $O/ladder_Raft_n3v2e3_hf1_compact.txt
[ $rc -eq 0 ] || [ $rc -eq 12 ] || [ $rc -eq 13 ] || exit $rc
timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -hostfrontier 1 -module Raft -config configs/Raft_n3v2e2.cfg > $O/bench_wl_hf1_compact.txt 2>&1; echo "bench-wl hf rc=$?"; tail -2 $O/bench_wl_hf1_compact.txt
