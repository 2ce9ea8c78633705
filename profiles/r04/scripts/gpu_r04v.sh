#!/bin/bash
# r04: logical shards write records and win flags straight into their owners'
# / generators' buffers (no copy for either exchange step): the sharded GPU
# tests, then 8 and 2 logical shards on the bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04v}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_order.py tests/test_gpu_sharded_mp.py "tests/test_gpu_configs.py::test_rung_two_logical_shards" "tests/test_gpu_configs.py::test_ladder_prefix_logical_shards" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --no-cpu-baseline --steps 3 > $O/bench_logical_$W.json 2> $O/bench_logical_$W.err || { echo "bench W=$W failed"; tail -5 $O/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_logical_$W.json')); print($W, d['ms_per_step'], d['kernel_ms'])"
done
