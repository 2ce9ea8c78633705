#!/bin/bash
# r04 k_expand A/B: CLI exhaustive checks of the bench workload, builds interleaved
# (each run = one fresh process, after a short idle so freed HBM has been cleared).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-ab_r04}
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for b in ${BUILDS:-build build_fast2 build_waves6}; do
    sleep 20
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg $CLI_ARGS > $O/$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/$b.$rep.txt; exit 1; }
    echo "$b rep$rep $(tail -1 $O/$b.$rep.txt)" >> $O/ab.txt
  done
done
cat $O/ab.txt | cut -c1-260
# counts of what the inserts do (RMC_FPSTATS build: inserts, 4-entry group loads, CAS issued / won, atomicMin)
if [ -x ./raft-tlaplus_amd/build_fpstats/raftmc ]; then
  sleep 20
  timeout -k 10 180 ./raft-tlaplus_amd/build_fpstats/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg > $O/fpstats.txt 2>&1 || { echo "fpstats failed"; tail -3 $O/fpstats.txt; exit 1; }
  grep -E "fingerprint-set inserts|fingerprint set:" $O/fpstats.txt
fi
