#!/bin/bash
# r04 A/B: parent rows staged only up to their last message (build_stage,
# -DRMC_STAGE_TRIM, k_expand and k_materialize) vs build -- CLI, fresh process,
# interleaved -- the parity suites on build_stage, and the kernel-trace stats
# of 8 logical shards on build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04u}; mkdir -p $O
: > $O/ab.txt
CFG="-deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2 3; do
  for b in build build_stage; do
    sleep 15
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc $CFG > $O/single.$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/single.$b.$rep.txt; exit 1; }
    echo "single $b rep$rep $(tail -1 $O/single.$b.$rep.txt)" >> $O/ab.txt
  done
done
cut -c1-300 $O/ab.txt
RAFTMC_BUILD=build_stage timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py tests/test_gpu_kraft.py tests/test_gpu_n5.py tests/test_gpu_variant2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_stage.log 2>&1 || { echo "stage tests failed"; tail -30 $O/pytest_stage.log; exit 1; }
tail -2 $O/pytest_stage.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt8 -o run --output-format csv -- python3 $R/bench.py --logical-shards 8 --no-cpu-baseline --steps 1 --warmup 1 > $O/kt8.log 2>&1 || { echo "kernel-trace failed"; tail -5 $O/kt8.log; exit 1; }
cp $(find $O/kt8 -name '*kernel_stats.csv' | head -1) $O/kernel_stats_logical8.csv
find $O/kt8 -name '*.csv' | xargs rm -f
