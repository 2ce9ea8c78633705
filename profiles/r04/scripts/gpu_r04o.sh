#!/bin/bash
# r04: the whole -m gpu suite on the current build, then the bench with and
# without the materialize/expand overlap, then 8 and 2 logical shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04o}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in 0 1 0 1; do
  RMC_NO_OVERLAP=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > $O/bench_noov$v.json 2> $O/bench_noov$v.err || { echo "bench $v failed"; tail -5 $O/bench_noov$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_noov$v.json')); print('no_overlap=$v', round(d['ms_per_step'],1), d['kernel_ms'], d['result']['distinct'])"
done
for W in 8 2; do
  RMC_VERBOSE=1 timeout -k 10 300 python -u bench.py --logical-shards $W --no-cpu-baseline --steps 2 > $O/bench_logical_$W.json 2> $O/bench_logical_$W.err || { echo "bench W=$W failed"; tail -5 $O/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_logical_$W.json')); print($W, d['ms_per_step'], d['kernel_ms'])"
  grep "HBM GiB: set" $O/bench_logical_$W.err | tail -$W
done
