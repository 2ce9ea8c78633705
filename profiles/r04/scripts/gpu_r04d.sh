#!/bin/bash
# r04: the logical-shard transport with batched copies: sharded tests, then
# the bench workload with W = 2 and 8 logical shards on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_mp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sharded.log 2>&1 || { echo "sharded tests failed"; tail -30 $O/pytest_sharded.log; exit 1; }
tail -2 $O/pytest_sharded.log
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --no-cpu-baseline --steps 2 > $O/bench_logical_$W.json 2> $O/bench_logical_$W.err || { echo "bench W=$W failed"; tail -5 $O/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_logical_$W.json')); print($W, d['ms_per_step'], d['kernel_ms'])"
done
