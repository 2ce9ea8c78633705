#!/bin/bash
# r03: parity subset on the vectorized-staging + growth-policy build, A/B and
# cold-process timing vs build_prev, bench, and config 2 with the host frontier
# from the start (-hostfrontier 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_configs.py tests/test_gpu_host_frontier.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
CFG=configs/Raft_n3v2e2.cfg
for i in 1 2; do
  for b in build build_prev; do
    sleep 30  # let the driver clear the previous process's HBM: a cold check, not a queued one
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config $CFG > $O/cold_${b}_$i.txt 2>&1 || { echo "$b failed"; exit 1; }
    echo "cold $b $(tail -1 $O/cold_${b}_$i.txt)"
  done
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
export RMC_HOST_FRONTIER_GIB=245
timeout -k 10 900 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -hostfrontier 1 -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_hf1.txt 2>&1; echo "cfg2 rc=$?"
grep -E "Error|states generated|depth of|Finished|host frontier:" $O/ladder_Raft_n3v2e3_hf1.txt | cut -c1-200
grep -E "^\[rmc\] depth (2[6-9]|3[0-9]):" $O/ladder_Raft_n3v2e3_hf1.txt | cut -c1-240
