#!/bin/bash
# FlexibleRaft.cfg (5 servers, BASELINE config 3) on one GPU, time-limited,
# per-level progress in gpurun_out/flex_probe.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${LIMIT:-240} ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module FlexibleRaft -config configs/FlexibleRaft.cfg > gpurun_out/flex_probe.txt 2>&1
rc=$?; echo "flex rc=$rc"; tail -4 gpurun_out/flex_probe.txt
