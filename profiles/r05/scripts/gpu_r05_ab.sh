#!/bin/bash
# r05: persistent k_expand (LDS-DMA prefetch of the next tile) -- the GPU suite
# on it, then the bench line interleaved with the one-tile-per-block build
# (build_np, -DRMC_EXPAND_PERSIST=0) for the A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05ab
O=gpurun_out/r05ab
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_persist.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest_persist.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for b in build build_np; do
    RAFTMC_BUILD=$b timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_${b}_$i.json 2> $O/bench_${b}_$i.err; rc=$?
    echo "$b #$i rc=$rc $(python -c "import json,sys; d=json.load(open('$O/bench_${b}_$i.json')); print(d['ms_per_step'], d['kernel_ms'], d['result']['first_check_s'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
