#!/bin/bash
# r04 closing measurements on the current build: the whole -m gpu suite, the
# profile set (tools/gpu_profile.sh: bench line, kernel-trace stats, FETCH /
# WRITE / SQ PMC passes, calibration), then 8 and 2 logical shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04s}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
TAG=r04 timeout -k 10 1000 bash tools/gpu_profile.sh > $O/profile.out 2>&1 || { echo "profile failed"; tail -20 $O/profile.out; exit 1; }
head -3 $O/profile.out | cut -c1-600
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --no-cpu-baseline --steps 2 > $O/bench_logical_$W.json 2> $O/bench_logical_$W.err || { echo "bench W=$W failed"; tail -5 $O/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_logical_$W.json')); print($W, d['ms_per_step'], d['kernel_ms'])"
done
