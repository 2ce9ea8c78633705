#!/bin/bash
# r05j: A/B of the XCD-aware block -> tile map (build_xcd: -DRMC_XCD_REMAP=1)
# against the default build on the bench workload, interleaved, bench.py's
# own timing (3 checks after a warm-up), counts checked
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
O=$R/gpurun_out/r05j
mkdir -p $O
for i in 1 2 3; do
  for b in build build_xcd; do
    if [ $b = build ]; then unset RAFTMC_BUILD; else export RAFTMC_BUILD=$b; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > $O/bench_${b}_$i.json 2> $O/bench_${b}_$i.err; rc=$?
    echo "$b #$i rc=$rc $(python -c "import json; d=json.loads(open('$O/bench_${b}_$i.json').read().strip().splitlines()[-1]); r=d['result']; print(round(d['ms_per_step'],1), r['distinct'], r['hidden_var_collisions'], {k: round(v,1) for k, v in d['kernel_ms'].items()})")"
    [ $rc -eq 0 ] || exit $rc
  done
done
