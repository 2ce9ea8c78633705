#!/bin/bash
# bench line + rocprofv3 kernel-trace summary of the same workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- $GRAFT_REPO_ROOT/raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config $GRAFT_REPO_ROOT/configs/${PROF_CFG:-Raft_n3v2e2}.cfg > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit $rc
