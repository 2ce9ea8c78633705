#!/bin/bash
# Parity tests, then the bench workload through the CLI (kernel ms in the JSON line).
# Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-Raft_n3v2e2}; do
  mod=$cfg; case $cfg in Raft_*) mod=Raft;; esac
  timeout -k 10 ${RUN_LIMIT:-200} ./raft-tlaplus_amd/build/raftmc -deadlock -json -module $mod -config configs/$cfg.cfg > gpurun_out/run_${TAG}_$cfg.txt 2>&1; rc=$?
  echo "$cfg rc=$rc"; tail -1 gpurun_out/run_${TAG}_$cfg.txt
  [ $rc -eq 0 ] || [ $rc -eq 12 ] || exit $rc
done
