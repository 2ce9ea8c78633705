#!/bin/bash
# r04 A/B: device rows written only up to their last message (build_trim,
# -DRMC_ROW_TRIM: the padding stores masked off) vs build -- CLI, fresh
# process, interleaved -- then the parity / order / sharded / host-frontier /
# checkpoint GPU tests on build_trim's library (RAFTMC_BUILD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04t}; mkdir -p $O
: > $O/ab.txt
CFG="-deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2 3; do
  for b in build build_trim; do
    sleep 15
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc $CFG > $O/single.$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/single.$b.$rep.txt; exit 1; }
    echo "single $b rep$rep $(tail -1 $O/single.$b.$rep.txt)" >> $O/ab.txt
  done
done
cut -c1-300 $O/ab.txt
RAFTMC_BUILD=build_trim timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py tests/test_gpu_checkpoint.py tests/test_gpu_kraft.py tests/test_gpu_simulate.py tests/test_gpu_n5.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_trim.log 2>&1 || { echo "trim tests failed"; tail -30 $O/pytest_trim.log; exit 1; }
tail -2 $O/pytest_trim.log
