#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the fingerprint-set insert in isolation
# (rmc_fpset_bench k_batch) at two duplicate mixes: ~all duplicates of an
# earlier level (no atomics expected) and ~all new keys (CAS + atomicMin each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for dup in 0.999 0.72 0.01; do
  for c in WRITE_SIZE FETCH_SIZE; do
    O=$R/gpurun_out/fpmc_${dup}_$c
    rm -rf $O
    timeout -s KILL 120 rocprofv3 --pmc $c -d $O -o run --output-format csv -- $R/raft-tlaplus_amd/build/fpset_bench -slots_log2 30 -batch 67108864 -dup $dup -loads 0.5 > $O.log 2>&1 || { echo "pmc failed"; exit 1; }
    python3 $R/tools/pmc_summary.py $O.json --pmc $(find $O -name '*counter_collection.csv' | head -1) > /dev/null
    python3 -c "
import json; d=json.load(open('$O.json'))
for k,v in d['kernels'].items():
    if 'k_batch' in k: print('dup $dup', '$c', '%.4g B per insert' % (v['${c}_per_dispatch']*1024/67108864))"
    grep '^{' $O.log | head -1
    rm -rf $O
  done
done
