#!/bin/bash
# r04: the TLA+ front end's lowered Next on the GPU (DuplicateMessage / DropMessage,
# reordered / reduced Next), then the whole -m gpu suite and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_frontend.log 2>&1 || { echo "frontend tests failed"; tail -30 $O/pytest_frontend.log; exit 1; }
tail -3 $O/pytest_frontend.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['kernel_ms'])"
