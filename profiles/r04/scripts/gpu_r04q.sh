#!/bin/bash
# r04 A/B (CLI, one fresh process per run, interleaved, 20 s idle before each):
#  single-GPU check of the bench workload with one stream (RMC_NO_OVERLAP=1,
#  kernel times comparable) -- build vs build_align4 (64 B aligned home groups);
#  8 logical shards -- build vs build_recv8 (8 records per owner thread) vs build_align4;
#  build_coherent: agent-scope (sc1) group loads; build_coh_fpstats counts its CAS / atomicMin;
#  fpset_bench at 2^24 / 2^28 / 2^32 slots (does the insert rate depend on the table's size?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04q}; mkdir -p $O
: > $O/ab.txt
CFG="-deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg"
for rep in 1 2; do
  for b in build build_align4 build_coherent; do
    sleep 15
    RMC_NO_OVERLAP=1 timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc $CFG > $O/single.$b.$rep.txt 2>&1 || { echo "$b failed"; tail -3 $O/single.$b.$rep.txt; exit 1; }
    echo "single $b rep$rep $(tail -1 $O/single.$b.$rep.txt)" >> $O/ab.txt
  done
done
for rep in 1 2; do
  for b in build build_recv8 build_align4 build_coherent; do
    sleep 15
    timeout -k 10 180 ./raft-tlaplus_amd/$b/raftmc $CFG -shards 8 > $O/w8.$b.$rep.txt 2>&1 || { echo "$b W=8 failed"; tail -3 $O/w8.$b.$rep.txt; exit 1; }
    echo "w8 $b rep$rep $(tail -1 $O/w8.$b.$rep.txt)" >> $O/ab.txt
  done
done
cut -c1-300 $O/ab.txt
RMC_NO_OVERLAP=1 timeout -k 10 180 ./raft-tlaplus_amd/build_coh_fpstats/raftmc $CFG -v > $O/coh_fpstats.txt 2>&1 || { echo "coh fpstats failed"; tail -3 $O/coh_fpstats.txt; exit 1; }
grep -E "fingerprint-set inserts" $O/coh_fpstats.txt
for s in 24 28 32; do
  timeout -k 10 120 ./raft-tlaplus_amd/build/fpset_bench -slots_log2 $s -dup 0.72 -loads 0.44 > $O/fpset_$s.txt 2>&1 || { echo "fpset_bench $s failed"; tail -3 $O/fpset_$s.txt; exit 1; }
  cat $O/fpset_$s.txt
done
