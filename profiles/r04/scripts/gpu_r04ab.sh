#!/bin/bash
# r04: k_expand phase costs on the final kernels (RMC_DIAG build): level 45's
# first chunk stopped after staging / bindings / deltas / fingerprints, and
# the real launch (tools/profile_expand.py), three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04ab}; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python3 -u tools/profile_expand.py build_diag 45 > $O/phases_$rep.json 2>&1 || { echo "phases failed"; tail -3 $O/phases_$rep.json; exit 1; }
  tail -1 $O/phases_$rep.json
done
