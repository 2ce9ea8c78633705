#!/bin/bash
# r06: config 5 chosen by measurement: the RaftFsync R-ladder
# at V=1, E=2, R = 3, 4, ... on one GPU (auto host frontier), until a rung no
# longer exhausts.  Each rung under its own time limit; logs to gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ladder5
B=raft-tlaplus_amd/build/raftmc
for R in 3 4 5 6 7; do
  cfg=configs/RaftFsync_n3v1e2r$R.cfg
  RMC_HOST_FRONTIER_GIB=240 timeout -k 10 420 $B -deadlock -v -json -module RaftFsync -config $cfg \
     > gpurun_out/ladder5/RaftFsync_n3v1e2r$R.txt 2>&1
  rc=$?
  echo "R=$R rc=$rc"; tail -4 gpurun_out/ladder5/RaftFsync_n3v1e2r$R.txt
  if [ $rc -ne 0 ] && [ $rc -ne 12 ] && [ $rc -ne 13 ]; then echo "stopping after R=$R (rc $rc)"; break; fi
  grep -q '"status":0' gpurun_out/ladder5/RaftFsync_n3v1e2r$R.txt || { echo "R=$R did not exhaust: the ladder ends here"; break; }
done
