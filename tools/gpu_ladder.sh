#!/bin/bash
# Scale ladder probe: each rung under its own time limit; stop on a dead step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in PullRaft RaftFsync Raft_n3v1e3 Raft_n3v2e2 Raft_n3v2e3; do
  mod=$cfg; case $cfg in Raft_*) mod=Raft;; esac
  timeout -k 10 ${RUNG_LIMIT:-240} ./raft-tlaplus_amd/build/raftmc -deadlock -json -v configs/$mod.tla -config configs/$cfg.cfg > gpurun_out/ladder_$cfg.txt 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/ladder_$cfg.txt
  [ $rc -eq 0 ] || [ $rc -eq 12 ] || [ $rc -eq 13 ] || [ $rc -eq 1 ] || exit $rc
done
