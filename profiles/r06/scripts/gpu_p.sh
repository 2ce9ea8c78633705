#!/bin/bash
# r06 (session 2): k_mark_tiles without the tile-dedup reference load (dedup off) and one phase-B block barrier fewer in k_expand (build_bar1) vs the committed kernels (build_bar0, 19d0f7c).
# Both RMC_DEV_ONE, same host objects.
# CLI on the bench workload, interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p
for round in 1 2 3; do
  for b in build_bar0 build_bar1; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/p/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/p/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/p/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/p/ab_mark_ref_barrier.txt || { echo "ab loop failed"; exit 1; }
