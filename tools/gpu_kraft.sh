#!/bin/bash
# KRaft on the GPU: the shipped cfg's constants through the CLI (per-level record), then the -m gpu KRaft tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module KRaft -config configs/KRaft.cfg > gpurun_out/kraft_cfg.txt 2>&1; rc=$?
echo "KRaft.cfg rc=$rc"; tail -4 gpurun_out/kraft_cfg.txt
[ $rc -eq 0 ] || [ $rc -eq 12 ] || [ $rc -eq 13 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kraft.py -m gpu -x -v --timeout 300 --timeout-method thread  > gpurun_out/pytest_kraft.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_kraft.log
exit $rc
