#!/bin/bash
# r03, A/B: k_materialize with rows staged in LDS and copied out whole-wave
# (build_stage, -DRMC_MAT_STAGE) against the default build, on the bench cfg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03k
mkdir -p $O
CFG=configs/Raft_n3v2e2.cfg
run() {  # build tag
  timeout -k 10 120 ./raft-tlaplus_amd/$1/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $CFG > $O/$2.txt 2>&1 || { echo "$1 failed"; tail -3 $O/$2.txt; exit 1; }
  echo "$1 $(tail -1 $O/$2.txt)"
}
for i in 1 2 3; do
  for b in build build_stage; do run $b ${b}_$i; done
done
cd /tmp && export TMPDIR=/tmp
for v in build build_stage; do
  for c in WRITE_SIZE FETCH_SIZE; do
    P=$O/pmc_${v}_$c
    timeout -s KILL 150 rocprofv3 --pmc $c -d $P -o run --output-format csv -- $R/raft-tlaplus_amd/$v/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $R/$CFG > $P.log 2>&1 || { echo "pmc $v $c failed"; tail -3 $P.log; exit 1; }
    F=$(find $P -name '*counter_collection.csv' | head -1)
    python3 $R/tools/pmc_summary.py $P.json --pmc $F > /dev/null
    python3 -c "
import json; d=json.load(open('$P.json'))
for k,v in sorted(d['kernels'].items()):
    if k.startswith('rmc::k_'): print('$v $c', k[:24], '%.4g MB/dispatch' % (v['${c}_per_dispatch']*1024/1e6), '%.3f ms' % (v['avg_ns']/1e6))"
    rm -rf $P
  done
done
cd $R
export RMC_HOST_FRONTIER_GIB=245
timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_auto.txt 2>&1; echo "cfg2 rc=$?"
grep -E "moved|host frontier:|depth 2[6-9]:" $O/ladder_Raft_n3v2e3_auto.txt | cut -c1-200
RMC_HF_PREPIN=32 timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e3.cfg > $O/ladder_Raft_n3v2e3_auto_prepin.txt 2>&1; echo "cfg2 prepin rc=$?"
grep -E "moved|host frontier:|depth 2[6-9]:" $O/ladder_Raft_n3v2e3_auto_prepin.txt | cut -c1-200
