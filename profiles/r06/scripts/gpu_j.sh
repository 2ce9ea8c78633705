#!/bin/bash
# r06 (session 2): tile-local dedup of the HBM inserts (one LDS round table,
# one barrier per 256-successor round, duplicates reference their
# representative's candidate) against the same tree without it (build_trim7).
# All RMC_DEV_ONE; CLI on the bench workload, interleaved; then the insert /
# atomic counts of the dedup build (RMC_FPSTATS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/j
for round in 1 2 3; do
  for b in build_trim7 build_dd; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/j/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/j/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/j/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/j/ab_tile_dedup.txt || { echo "ab loop failed"; exit 1; }
timeout -k 10 200 raft-tlaplus_amd/build_ddstats/raftmc -deadlock -v -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/j/fpstats_dedup.txt 2>&1 || { echo "fpstats failed"; tail -5 gpurun_out/j/fpstats_dedup.txt; exit 1; }
grep -E "fingerprint-set inserts|Finished|generated" gpurun_out/j/fpstats_dedup.txt
