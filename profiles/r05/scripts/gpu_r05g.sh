#!/bin/bash
# r05g: config 3 (FlexibleRaft.cfg verbatim, N = 5) on 4 logical shards, each
# shard's levels in host pages, as deep as the host allows -- to compare every
# level with the single-GPU host-frontier ladder (profiles/r03/ladder_FlexibleRaft_hf1.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
O=$R/gpurun_out/r05g
mkdir -p $O
timeout -k 10 400 $R/raft-tlaplus_amd/build/raftmc -deadlock -json -v -shards 4 -hostfrontier 1 -module FlexibleRaft -config $R/configs/FlexibleRaft.cfg > $O/flex_cfg3_shards4_hf1.txt 2>&1; rc=$?
echo "FlexibleRaft.cfg -shards 4 -hostfrontier 1 rc=$rc $(tail -n 1 $O/flex_cfg3_shards4_hf1.txt)"
exit 0
