#!/bin/bash
# r06 (session 2): action-major phase C lanes (RMC_ACT_MAJOR) against the same
# tree parent-major (build_trim7).  All RMC_DEV_ONE; CLI on the bench
# workload, interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/k
for round in 1 2 3; do
  for b in build_trim7 build_am; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/k/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/k/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/k/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/k/ab_act_major.txt || { echo "ab loop failed"; exit 1; }
