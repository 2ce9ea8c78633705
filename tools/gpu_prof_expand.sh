#!/bin/bash
# k_expand phase decomposition (tools/profile_expand.py) for each RMC_DIAG build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_expand
for b in ${BUILDS:-build_diag}; do
  for L in ${LEVELS:-45}; do
    timeout -k 10 120 python3 -u tools/profile_expand.py $b $L >> gpurun_out/prof_expand/phases.jsonl 2> gpurun_out/prof_expand/$b.err || { echo "$b failed"; tail -5 gpurun_out/prof_expand/$b.err; exit 1; }
  done
done
cat gpurun_out/prof_expand/phases.jsonl
