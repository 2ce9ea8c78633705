#!/bin/bash
# r06 (session 2): A/B of the batched staging (RMC_STAGE_BATCH): every load of
# a thread issued before its first LDS write in k_expand phase A and
# k_materialize, k_mark_tiles wave-local with its candidate loads unconditional.
# build_ts1 adds fixed per-tile candidate slots (RMC_TILE_SLOTS). All builds are RMC_DEV_ONE (Raft N=3 only), same host objects; CLI on the
# bench workload, interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f
for round in 1 2 3; do
  for b in build_sb0 build_sb1 build_ts1; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/f/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/f/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/f/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/f/ab_stage_batch.txt || { echo "ab loop failed"; exit 1; }
