#!/bin/bash
# r06 (session 2): phase-B barriers: build_bar0 = 19d0f7c, build_bar1 = one wave-0 barrier replaced by a wave sync (+ no REF load in k_mark_tiles), build_bar2 = + per-wave chunk tables (no block barrier between the guard masks and the chunk loop).
# Both RMC_DEV_ONE, same host objects.
# CLI on the bench workload, interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
for round in 1 2 3; do
  for b in build_bar0 build_bar1 build_bar2; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/q/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/q/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/q/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/q/ab_phase_b_barriers.txt || { echo "ab loop failed"; exit 1; }
