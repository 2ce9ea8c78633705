#!/bin/bash
# r04 A/B: the lost-CAS path's atomicMin issued without first reading the
# value (build_blindmin, -DRMC_FP_BLINDMIN) vs build (CLI, fresh process,
# interleaved, 15 s idle before each), and its RMC_FPSTATS counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04r}; mkdir -p $O
: > $O/ab.txt
CFG="-deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2 3; do
  for b in build build_blindmin; do
    sleep 15
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc $CFG > $O/single.$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/single.$b.$rep.txt; exit 1; }
    echo "single $b rep$rep $(tail -1 $O/single.$b.$rep.txt)" >> $O/ab.txt
  done
done
cut -c1-300 $O/ab.txt
timeout -k 10 180 ./raft-tlaplus_amd/build_bm_fpstats/raftmc $CFG -v > $O/bm_fpstats.txt 2>&1 || { echo "bm fpstats failed"; tail -3 $O/bm_fpstats.txt; exit 1; }
grep -E "fingerprint-set inserts" $O/bm_fpstats.txt
