#!/bin/bash
# rocprofv3 kernel-trace summary of the bench command (per-kernel time):
# gpurun_out/kstats_$TAG.csv.  One GPU step, time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-ks}
O=$R/gpurun_out/kst_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps ${STEPS:-2} --warmup 1 $BENCH_ARGS > $O/bench.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -2 $O/bench.log
f=$(find $O -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp $f $R/gpurun_out/kstats_$TAG.csv && cut -d, -f1-8 $f | head -20
find $O -name '*kernel_trace.csv' -o -name '*agent_info.csv' | xargs rm -f
exit $rc
