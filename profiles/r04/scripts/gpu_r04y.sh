#!/bin/bash
# r04 A/B: a lane's share of its parent's message sums / live masks kept in
# registers and published with one LDS atomic per word (build_sumsreg,
# -DRMC_SUMS_REG) vs build -- CLI, fresh process, interleaved -- then the
# parity / order / n5 / sharded suites on build_sumsreg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04y}; mkdir -p $O
: > $O/ab.txt
CFG="-deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2 3; do
  for b in build build_sumsreg; do
    sleep 15
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc $CFG > $O/single.$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/single.$b.$rep.txt; exit 1; }
    echo "single $b rep$rep $(tail -1 $O/single.$b.$rep.txt)" >> $O/ab.txt
  done
done
cut -c1-300 $O/ab.txt
RAFTMC_BUILD=build_sumsreg timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_n5.py tests/test_gpu_sharded.py tests/test_gpu_kraft.py tests/test_gpu_variant2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sr.log 2>&1 || { echo "sr tests failed"; tail -30 $O/pytest_sr.log; exit 1; }
tail -2 $O/pytest_sr.log
