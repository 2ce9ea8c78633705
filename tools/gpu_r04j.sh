#!/bin/bash
# r04: logical shards write winners straight into their owners' rows (piece
# map): sharded / host-frontier / configs GPU tests, then the bench workload
# on 8 and 2 logical shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04j}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py tests/test_gpu_configs.py tests/test_gpu_sharded_mp.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=8 > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --no-cpu-baseline --steps 2 > $O/bench_logical_$W.json 2> $O/bench_logical_$W.err || { echo "bench W=$W failed"; tail -5 $O/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_logical_$W.json')); print($W, d['ms_per_step'], d['kernel_ms'])"
done
