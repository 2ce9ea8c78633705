#!/bin/bash
# r06 (session 2): the whole -m gpu suite on the batched-staging + tile-slot
# build, smoke, then the profile (bench line, kernel trace, PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/g/pytest_g.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" gpurun_out/g/pytest_g.log | head -20; tail -30 gpurun_out/g/pytest_g.log; exit 1; }
tail -2 gpurun_out/g/pytest_g.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g/smoke_g.log 2>&1 || { echo smoke failed; cat gpurun_out/g/smoke_g.log; exit 1; }
cat gpurun_out/g/smoke_g.log
TAG=r06s2 bash tools/gpu_profile.sh
