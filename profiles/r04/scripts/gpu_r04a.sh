#!/bin/bash
# r04 first check: smoke, the changed tests first (checkpoint / host frontier /
# ABI), then the whole -m gpu suite and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04a}
mkdir -p $O
timeout -k 10 240 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_checkpoint.py tests/test_gpu_host_frontier.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_changed.log 2>&1 || { echo "changed tests failed"; tail -30 $O/pytest_changed.log; exit 1; }
tail -3 $O/pytest_changed.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
