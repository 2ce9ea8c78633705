#!/bin/bash
# r06 second GPU pass: the whole -m gpu suite on the compiled-handler build,
# smoke, then the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/pytest_b.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" gpurun_out/pytest_b.log | head -20; tail -30 gpurun_out/pytest_b.log; exit 1; }
tail -2 gpurun_out/pytest_b.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_b.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke_b.log; exit 1; }
cat gpurun_out/smoke_b.log
timeout -k 10 300 python bench.py > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { echo "bench failed"; tail -20 gpurun_out/bench_b.err; exit 1; }
cat gpurun_out/bench_b.json
