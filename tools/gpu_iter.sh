#!/bin/bash
# One iteration on the GPU box: the -m gpu suite (or TESTS=...), the bench line
# (no CPU baseline unless CPU=1), and optional CLI runs (RUNS="Raft_n3v2e2 ...").
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-it}
if [ "${TESTS:-all}" != "none" ]; then
  sel=${TESTS:-tests}; [ "$sel" = all ] && sel=tests
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  cpu="--no-cpu-baseline"; [ "${CPU:-0}" = 1 ] && cpu=""
  timeout -k 10 ${BENCH_LIMIT:-400} python -u bench.py $cpu $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
  [ $rc -eq 0 ] || exit $rc
fi
for cfg in $RUNS; do
  mod=$cfg; case $cfg in Raft_*) mod=Raft;; PullRaft_*) mod=PullRaft;; RaftFsync_*) mod=RaftFsync;; FlexibleRaft_*) mod=FlexibleRaft;; KRaft_*) mod=KRaft;; esac
  timeout -k 10 ${RUN_LIMIT:-240} ./raft-tlaplus_amd/build/raftmc -deadlock -json -v $RUN_ARGS -module $mod -config configs/$cfg.cfg > gpurun_out/run_${TAG}_$cfg.txt 2>&1; rc=$?
  echo "$cfg rc=$rc"; tail -2 gpurun_out/run_${TAG}_$cfg.txt
  [ $rc -eq 0 ] || [ $rc -eq 12 ] || [ $rc -eq 13 ] || exit $rc
done
exit 0
