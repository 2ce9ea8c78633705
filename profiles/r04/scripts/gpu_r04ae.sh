#!/bin/bash
# r04: BASELINE config 2 (Raft_n3v2e3) on 2 logical shards with per-shard
# host frontiers, to depth 29 -- the sharded capacity path at scale; its
# counts must equal the single-GPU host-frontier ladder's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04ae}; mkdir -p $O
timeout -k 10 400 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -shards 2 -hostfrontier 1 -maxdepth 29 -module Raft -config configs/Raft_n3v2e3.cfg > $O/cfg2_shards2_hf1.txt 2>&1 || { echo "run failed"; tail -5 $O/cfg2_shards2_hf1.txt; exit 1; }
grep -E "depth 2[5-9]|shard . HBM" $O/cfg2_shards2_hf1.txt | cut -c1-250
tail -1 $O/cfg2_shards2_hf1.txt
