#!/bin/bash
# r04: (1) when released VMM chunks' HBM comes back (tools/probe/vmm_free_probe);
# (2) the k_expand A/B builds + RMC_FPSTATS counts (tools/gpu_ab_r04.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04n}; mkdir -p $O
timeout -k 10 120 ./tools/probe/vmm_free_probe > $O/vmm_free_probe.txt 2>&1; echo "probe rc=$?"; cat $O/vmm_free_probe.txt
TAG=ab_r04 timeout -k 10 900 bash tools/gpu_ab_r04.sh
