#!/bin/bash
# Scale ladder probe: each rung under its own time limit; stop at the first
# rung that does not finish cleanly (no further GPU step after a timeout).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${RUNGS:-PullRaft RaftFsync Raft_n3v1e3 FlexibleRaft Raft_n3v2e3}; do
  mod=$cfg; case $cfg in Raft_*) mod=Raft;; esac
  timeout -k 10 ${RUNG_LIMIT:-180} ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module $mod -config configs/$cfg.cfg > gpurun_out/ladder_$cfg.txt 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/ladder_$cfg.txt
  echo "$cfg rc=$rc"; grep -E "^\{|Error|capacity" gpurun_out/ladder_$cfg.txt | head -3
  [ $rc -eq 0 ] || [ $rc -eq 12 ] || exit $rc
done
