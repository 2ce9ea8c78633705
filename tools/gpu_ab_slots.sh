#!/bin/bash
# A/B: k_expand / k_mark / k_materialize time of the bench workload (CLI, one
# cold process per run) at fixed fingerprint-set sizes (SLOTS="2^a ..." as log2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-Raft_n3v2e2}
for lg in ${SLOTS:-32 33}; do
  timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -hashslots $((1 << lg)) $ARGS -module Raft -config configs/$CFG.cfg > gpurun_out/ab_slots_$lg.txt 2>&1; rc=$?
  echo "slots 2^$lg rc=$rc: $(tail -1 gpurun_out/ab_slots_$lg.txt)"
  [ $rc -eq 0 ] || exit $rc
done
