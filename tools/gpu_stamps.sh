#!/bin/bash
# k_expand phase shares (diagnostic -DRMC_STAMPS build in build_st) on the bench cfg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-Raft_n3v2e2}
timeout -k 10 120 ./raft-tlaplus_amd/build_st/raftmc -deadlock -json -v -hashslots 4294967296 -module Raft -config configs/$CFG.cfg > gpurun_out/stamps.txt 2>&1; rc=$?
grep -E "phase shares|fingerprint set:" gpurun_out/stamps.txt; tail -1 gpurun_out/stamps.txt
exit $rc
