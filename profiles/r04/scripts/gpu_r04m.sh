#!/bin/bash
# r04: tests/test_gpu_configs.py's checks in order with free HBM after each (tools/hf_dbg.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04m}; mkdir -p $O
timeout -k 10 500 python -u tools/hf_dbg.py > $O/hf_dbg.txt 2>&1; echo "rc=$?"; grep -v "^\[rmc\] depth" $O/hf_dbg.txt | tail -40
