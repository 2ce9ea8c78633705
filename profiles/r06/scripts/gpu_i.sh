#!/bin/bash
# r06 (session 2): k_expand LDS trim (live-message mask of (kmax+31)/32 words,
# 16-bit tile prefix: 20.4 KB per block, eight blocks per CU) at 7 and at 8
# waves per SIMD (64 VGPRs, 48 B of scratch), against the untrimmed build.
# All RMC_DEV_ONE, same host objects; CLI on the bench workload, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/i
for round in 1 2 3; do
  for b in build_new build_trim7 build_trim8; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/i/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/i/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/i/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/i/ab_lds_trim.txt || { echo "ab loop failed"; exit 1; }
