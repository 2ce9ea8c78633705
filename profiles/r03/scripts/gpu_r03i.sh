#!/bin/bash
# r03: capacity runs with the levels on the host from the start, and an A/B of
# 256-thread k_materialize blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03i
mkdir -p $O
CFG=configs/Raft_n3v2e2.cfg
for i in 1 2; do
  for b in build build_mt256; do
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $CFG > $O/ab_${b}_$i.txt 2>&1 || { echo "$b failed"; exit 1; }
    echo "$b $(tail -1 $O/ab_${b}_$i.txt)"
  done
done
export RMC_HOST_FRONTIER_GIB=245
for c in KRaft:KRaft_n3v3e2 RaftFsync:RaftFsync_n3v2e2r1 FlexibleRaft:FlexibleRaft; do
  mod=${c%%:*}; cfg=${c##*:}
  timeout -k 10 600 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -hostfrontier 1 -module $mod -config configs/$cfg.cfg > $O/ladder_${cfg}_hf1.txt 2>&1; echo "$cfg rc=$?"
  grep -E "Error|states generated|depth of|Finished|^\{" $O/ladder_${cfg}_hf1.txt | cut -c1-220
done
