#!/bin/bash
# r04: capacity exhaustion in the sharded search ends with status 3 and the
# completed levels: the sharded / host-frontier GPU tests (incl. the new
# host-pages-exhausted test), then config 2 on 2 logical shards with host
# frontiers to depth 31 (host pages run out during level 31).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04ag}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -shards 2 -hostfrontier 1 -maxdepth 31 -module Raft -config configs/Raft_n3v2e3.cfg > $O/cfg2_shards2_hf1_d31.txt 2>&1; echo "raftmc rc=$?"
grep -E "depth (29|3[01])|shard . HBM|capacity" $O/cfg2_shards2_hf1_d31.txt | cut -c1-250
tail -1 $O/cfg2_shards2_hf1_d31.txt
