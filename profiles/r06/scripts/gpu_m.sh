#!/bin/bash
# r06 (session 2): apply_delta merge batched (RMC_MERGE_BATCH: the wave max message count, four LDS reads per block) vs the loop form.
# Both RMC_DEV_ONE, same host objects.
# CLI on the bench workload, interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/m
for round in 1 2 3; do
  for b in build_mb0 build_mb1; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/m/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/m/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/m/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/m/ab_merge_batch.txt || { echo "ab loop failed"; exit 1; }
