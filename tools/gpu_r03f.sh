#!/bin/bash
# r03: SQ/TCC counter passes (one pass per run, within the per-block limits)
# for the bench workload's kernels, summarised per kernel per dispatch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BIN=$R/raft-tlaplus_amd/${BUILD:-build}/raftmc
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
            "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ" ${EXTRA_PASSES}; do
  i=$((i+1))
  P=$O/pass$i
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $P -o run --output-format csv -- $BIN -deadlock -json -hashslots 4294967296 -module Raft -config $R/configs/Raft_n3v2e2.cfg > $P.log 2>&1 || { echo "pass $i failed"; tail -3 $P.log; exit 1; }
  F=$(find $P -name '*counter_collection.csv' | head -1)
  python3 $R/tools/pmc_summary.py $O/pass$i.json --pmc $F > /dev/null
  python3 - <<PY
import json
d=json.load(open('$O/pass$i.json'))
for k,v in sorted(d['kernels'].items()):
    if k.startswith('rmc::k_'):
        print(k[:24], ' '.join('%s=%.4g' % (c.replace('_per_dispatch',''), x) for c,x in sorted(v.items()) if c.endswith('_per_dispatch')))
PY
  rm -rf $P
done
