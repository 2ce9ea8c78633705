#!/bin/bash
# The sharded protocol's cost on one GPU: bench lines with W logical shards
# (SHARDS="1 2 8"), the single-shard path beside them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${SHARDS:-1 2 8}; do
  timeout -k 10 ${LIMIT:-300} python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --logical-shards $w $BENCH_ARGS > gpurun_out/shards_$w.json 2> gpurun_out/shards_$w.err; rc=$?
  echo "W=$w rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/shards_$w.json')); print(d['ms_per_step'], d['result']['distinct'], d['kernel_ms'])" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
