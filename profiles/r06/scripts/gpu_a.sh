#!/bin/bash
# r06 first GPU pass: the new multi-GPU front door, host-frontier regrowth,
# widening traces, then the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_multi.py tests/test_gpu_host_frontier.py tests/test_gpu_widen.py tests/test_gpu_checkpoint.py \
  > gpurun_out/pytest_a.log 2>&1 || { echo "pytest failed rc=$?"; tail -50 gpurun_out/pytest_a.log; exit 1; }
tail -3 gpurun_out/pytest_a.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { echo "bench failed"; tail -20 gpurun_out/bench_a.err; exit 1; }
cat gpurun_out/bench_a.json
