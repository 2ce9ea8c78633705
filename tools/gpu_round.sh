#!/bin/bash
# One gpurun call covering a build: smoke, the whole -m gpu suite, the bench
# line, and a rocprofv3 kernel-trace summary of the bench workload.  Each GPU
# step has its own time limit; the script stops at the first step that fails.
#   TAG=r03a tools/gpu_round.sh        (SKIP_TESTS=1 / SKIP_PROF=1 to drop steps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-r03}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 240 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -z "$SKIP_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $R/raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config $R/configs/${PROF_CFG:-Raft_n3v2e2}.cfg > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
  find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
  head -8 $O/kernel_stats.csv
fi
