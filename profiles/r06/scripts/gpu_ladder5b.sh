#!/bin/bash
# r06: the RaftFsync R-ladder at V=1, E=2 saturates at R=3 (1,179,899,717
# distinct for every R >= 3: restartCtr is outside VIEW).  The rungs between
# it and the V=2 / E=3 rungs with a restart: V=2, E=2, R=0 and V=1, E=3, R=0.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ladder5
B=raft-tlaplus_amd/build/raftmc
for c in RaftFsync_n3v2e2 RaftFsync_n3v1e3; do
  RMC_HOST_FRONTIER_GIB=240 timeout -k 10 480 $B -deadlock -v -json -module RaftFsync -config configs/$c.cfg \
     > gpurun_out/ladder5/$c.txt 2>&1
  rc=$?
  echo "$c rc=$rc"; tail -4 gpurun_out/ladder5/$c.txt
  if [ $rc -ne 0 ] && [ $rc -ne 12 ] && [ $rc -ne 13 ]; then echo "stopping (rc $rc)"; break; fi
done
