#!/bin/bash
# r03, third call: device-allocation costs (cold check), A/B of the insert
# protocol / tile dedup builds, PMC traffic per kernel, the k_expand phase
# decomposition with per-dispatch WRITE_SIZE, and two host-frontier ladders.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03c
mkdir -p $O
CFG=configs/Raft_n3v2e2.cfg
timeout -k 10 120 ./tools/probe/alloc_probe 64 > $O/alloc_probe.txt 2>&1 || { echo "alloc probe failed"; tail -5 $O/alloc_probe.txt; exit 1; }
cat $O/alloc_probe.txt
run() {  # build tag
  timeout -k 10 120 ./raft-tlaplus_amd/$1/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $CFG > $O/$2.txt 2>&1 || { echo "$1 failed"; tail -3 $O/$2.txt; exit 1; }
  echo "$1 $(tail -1 $O/$2.txt)"
}
for i in 1 2; do
  for b in build build_legacy build_nodedup build_r02; do run $b ${b}_$i; done
done
cd /tmp && export TMPDIR=/tmp
for v in build build_r02; do
  for c in WRITE_SIZE FETCH_SIZE; do
    P=$O/pmc_${v}_$c
    timeout -s KILL 150 rocprofv3 --pmc $c -d $P -o run --output-format csv -- $R/raft-tlaplus_amd/$v/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $R/$CFG > $P.log 2>&1 || { echo "pmc $v $c failed"; tail -3 $P.log; exit 1; }
    F=$(find $P -name '*counter_collection.csv' | head -1)
    python3 $R/tools/pmc_summary.py $P.json --pmc $F > /dev/null
    python3 -c "
import json; d=json.load(open('$P.json'))
for k,v in sorted(d['kernels'].items()):
    if k.startswith('rmc::k_'): print('$v $c', k, '%.4g MB/dispatch' % (v['${c}_per_dispatch']*1024/1e6))"
    rm -rf $P
  done
done
P=$O/pmc_diag_WRITE_SIZE
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $P -o run --output-format csv -- /usr/bin/python3 $R/tools/profile_expand.py build_diag 45 > $P.log 2>&1 || { echo "pmc diag failed"; tail -3 $P.log; exit 1; }
F=$(find $P -name '*counter_collection.csv' | head -1)
python3 $R/tools/pmc_dispatches.py $F k_expand > $O/diag_expand_dispatches.txt
grep -A0 "" $P.log | tail -2
rm -rf $P
cd $R
timeout -k 10 120 python3 -u tools/profile_expand.py build_diag 45 > $O/phases.json 2>&1 || { echo "phases failed"; tail -3 $O/phases.json; exit 1; }
cat $O/phases.json
export RMC_HOST_FRONTIER_GIB=240
timeout -k 10 400 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module RaftFsync -config configs/RaftFsync_n3v2e2r1.cfg > $O/ladder_fsync_n3v2e2r1_hf.txt 2>&1; echo "fsync rc=$?"
tail -5 $O/ladder_fsync_n3v2e2r1_hf.txt | cut -c1-300
timeout -k 10 400 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module KRaft -config configs/KRaft_n3v3e2.cfg > $O/ladder_kraft_n3v3e2_hf.txt 2>&1; echo "kraft rc=$?"
tail -5 $O/ladder_kraft_n3v3e2_hf.txt | cut -c1-300
