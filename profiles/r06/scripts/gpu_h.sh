#!/bin/bash
# r06 (session 2): A/B of global-typed row stores in k_materialize (global_store
# instead of flat_store: a flat store also counts in lgkmcnt, so every LDS wait
# after one waited for the store).  build_old = the committed kernels (f63ffba),
# build_new = this tree; both RMC_DEV_ONE, same host objects; CLI, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/h
for round in 1 2 3; do
  for b in build_old build_new; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/h/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/h/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/h/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/h/ab_global_rows.txt || { echo "ab loop failed"; exit 1; }
