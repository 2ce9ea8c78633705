#!/bin/bash
# r06 (session 2): k_mark_tiles with an LDS candidate-to-parent map (RMC_MARK_MAP=1024, build_mm1) vs the binary search (build_mm0).
# Both RMC_DEV_ONE, same host objects.
# CLI on the bench workload, interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t
for round in 1 2 3; do
  for b in build_mm0 build_mm1; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/t/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/t/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/t/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/t/ab_mark_map.txt || { echo "ab loop failed"; exit 1; }
