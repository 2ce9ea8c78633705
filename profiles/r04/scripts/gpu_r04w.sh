#!/bin/bash
# r04 A/B: wave-level dedup of equal fingerprints before the HBM probe
# (build_wdedup, -DRMC_WAVE_DEDUP) vs build -- CLI, fresh process,
# interleaved; its RMC_FPSTATS counts; 8 logical shards; then the parity /
# order / sharded / host-frontier / n5 / KRaft suites on build_wdedup.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04w}; mkdir -p $O
: > $O/ab.txt
CFG="-deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2 3; do
  for b in build build_wdedup; do
    sleep 15
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc $CFG > $O/single.$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/single.$b.$rep.txt; exit 1; }
    echo "single $b rep$rep $(tail -1 $O/single.$b.$rep.txt)" >> $O/ab.txt
  done
done
for rep in 1 2; do
  for b in build build_wdedup; do
    sleep 15
    timeout -k 10 180 ./raft-tlaplus_amd/$b/raftmc $CFG -shards 8 > $O/w8.$b.$rep.txt 2>&1 || { echo "$b W=8 failed"; tail -3 $O/w8.$b.$rep.txt; exit 1; }
    echo "w8 $b rep$rep $(tail -1 $O/w8.$b.$rep.txt)" >> $O/ab.txt
  done
done
cut -c1-300 $O/ab.txt
timeout -k 10 180 ./raft-tlaplus_amd/build_wd_fpstats/raftmc $CFG -v > $O/wd_fpstats.txt 2>&1 || { echo "wd fpstats failed"; tail -3 $O/wd_fpstats.txt; exit 1; }
grep -E "fingerprint-set inserts" $O/wd_fpstats.txt
RAFTMC_BUILD=build_wdedup timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py tests/test_gpu_kraft.py tests/test_gpu_n5.py tests/test_gpu_variant2.py "tests/test_gpu_configs.py::test_rung_exhaustive_record" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_wd.log 2>&1 || { echo "wd tests failed"; tail -30 $O/pytest_wd.log; exit 1; }
tail -2 $O/pytest_wd.log
