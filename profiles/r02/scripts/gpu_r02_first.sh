#!/bin/bash
# Round-2 first GPU call: the whole -m gpu suite, then the two BASELINE
# configs never run in round 1 (config 3 FlexibleRaft.cfg, config 2
# Raft_n3v2e3) through the CLI with per-level progress.  Each GPU step has its
# own time limit; the script stops at the first step that dies.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-540} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r02a.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${RUNGS:-FlexibleRaft Raft_n3v2e3}; do
  mod=$cfg; case $cfg in Raft_*) mod=Raft;; esac
  timeout -k 10 ${RUNG_LIMIT:-200} ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module $mod -config configs/$cfg.cfg > gpurun_out/ladder_r02_$cfg.txt 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/ladder_r02_$cfg.txt
  echo "$cfg rc=$rc"; tail -4 gpurun_out/ladder_r02_$cfg.txt
  [ $rc -eq 0 ] || [ $rc -eq 12 ] || [ $rc -eq 13 ] || [ $rc -eq 124 ] || exit $rc
  [ $rc -eq 124 ] && exit $rc
done
exit 0
