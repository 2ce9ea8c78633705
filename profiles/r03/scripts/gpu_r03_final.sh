#!/bin/bash
# r03 final: smoke, the whole -m gpu suite, then tools/gpu_profile.sh (bench
# line, kernel-trace stats of the bench command, FETCH/WRITE/SQ PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03_final
mkdir -p $O
timeout -k 10 240 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TAG=r03 timeout -k 10 1000 tools/gpu_profile.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -20 $O/profile.log; exit 1; }
tail -30 $O/profile.log
