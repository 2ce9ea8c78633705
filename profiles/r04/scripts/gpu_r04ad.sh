#!/bin/bash
# r04: what a fresh process's first check costs vs its message capacity:
# the CLI (one check per process, 15 s idle before each) with the default
# capacity (8N+8V+4E = 48 slots -> 256 B rows), -msgcap 35 (192 B rows: the
# bench's warm checks) and -msgcap 40, -v for the growth/setup lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04ad}; mkdir -p $O
: > $O/cold.txt
CFG="-deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2; do
  for k in 0 35 40; do
    sleep 15
    A=""; [ $k -gt 0 ] && A="-msgcap $k"
    timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc $CFG $A > $O/cold_$k.$rep.txt 2>&1 || { echo "K=$k failed"; tail -3 $O/cold_$k.$rep.txt; exit 1; }
    echo "K=$k rep$rep $(grep -E 'setup' $O/cold_$k.$rep.txt | cut -c1-120) $(tail -1 $O/cold_$k.$rep.txt)" >> $O/cold.txt
  done
done
cut -c1-400 $O/cold.txt
