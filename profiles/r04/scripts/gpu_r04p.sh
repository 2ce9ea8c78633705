#!/bin/bash
# r04: what the inserts do (RMC_FPSTATS build: inserts, group loads, CAS issued
# / won, atomicMin), then the r04 profile set (tools/gpu_profile.sh: bench,
# kernel-trace stats, FETCH/WRITE/SQ PMC passes, counter calibration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/r04p; mkdir -p $O
timeout -k 10 180 ./raft-tlaplus_amd/build_fpstats/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg > $O/fpstats.txt 2>&1 || { echo "fpstats failed"; tail -3 $O/fpstats.txt; exit 1; }
grep -E "fingerprint-set inserts|fingerprint set:|expand_ms" $O/fpstats.txt | cut -c1-400
TAG=r04 timeout -k 10 1000 bash tools/gpu_profile.sh
