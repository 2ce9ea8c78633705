#!/bin/bash
# A/B of builds (BUILDS="build build_b"): CLI timing of the bench cfg (HIP-event
# kernel ms), then one rocprofv3 --pmc pass per build (PMC="WRITE_SIZE" or
# "FETCH_SIZE"), summarised per kernel into gpurun_out/abpmc_<build>.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
CFG=${CFG:-Raft_n3v2e2}
for v in ${BUILDS:-build build_b}; do
  timeout -k 10 120 ./raft-tlaplus_amd/$v/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config configs/$CFG.cfg > gpurun_out/ab_$v.txt 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_$v.txt)"
done
for v in ${BUILDS:-build build_b}; do
  timeout -k 10 120 ./raft-tlaplus_amd/$v/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config configs/$CFG.cfg > gpurun_out/ab2_$v.txt 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab2_$v.txt)"
done
cd /tmp && export TMPDIR=/tmp
for v in ${BUILDS:-build build_b}; do
  for c in ${PMC:-WRITE_SIZE}; do
    O=$R/gpurun_out/abpmc_${v}_$c
    rm -rf $O
    timeout -s KILL 120 rocprofv3 --pmc $c -d $O -o run --output-format csv -- $R/raft-tlaplus_amd/$v/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $R/configs/$CFG.cfg > $O.log 2>&1 || { echo "pmc $v $c failed"; exit 1; }
    python3 $R/tools/pmc_summary.py $O.json --pmc $(find $O -name '*counter_collection.csv' | head -1) > /dev/null
    python3 -c "
import json; d=json.load(open('$O.json'))
for k,v in d['kernels'].items():
    if k.startswith('rmc::k_'): print('$v', '$c', k, '%.4g MB/dispatch' % (v['${c}_per_dispatch']*1024/1e6))"
    rm -rf $O
  done
done
