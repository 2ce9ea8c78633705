#!/bin/bash
# r06 third GPU pass: the config-5 R-ladder tests and the compiled-handler
# GPU tests on this build, RaftFsync_n3v2e2 (the node-sized config-5
# candidate) on 4 logical shards with host frontiers, then the r06 profile
# (bench line, kernel trace, PMC passes: tools/gpu_profile.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_handlers.py "tests/test_gpu_configs.py::test_fsync_r3_exhausts_and_its_prefix_equals_the_c_oracle" \
  "tests/test_gpu_configs.py::test_fsync_r_ladder_saturates" > gpurun_out/c/pytest_c.log 2>&1 \
  || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" gpurun_out/c/pytest_c.log | head -20; tail -30 gpurun_out/c/pytest_c.log; exit 1; }
tail -2 gpurun_out/c/pytest_c.log
RMC_HOST_FRONTIER_GIB=240 timeout -k 10 420 raft-tlaplus_amd/build/raftmc -deadlock -v -json -shards 4 -hostfrontier 1 \
  -maxdepth 36 -module RaftFsync -config configs/RaftFsync_n3v2e2.cfg > gpurun_out/c/RaftFsync_n3v2e2_shards4_hf1.txt 2>&1
rc=$?
echo "shards4 rc=$rc"; tail -5 gpurun_out/c/RaftFsync_n3v2e2_shards4_hf1.txt
if [ $rc -ne 0 ] && [ $rc -ne 12 ] && [ $rc -ne 13 ]; then echo "stopping (rc $rc)"; exit 1; fi
TAG=r06 bash tools/gpu_profile.sh
