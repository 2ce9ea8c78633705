#!/bin/bash
# r03: the capacity ladders in the default auto mode after the level-boundary
# switch, threaded pinning and split copy streams (compare the *_hf1 runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03p
mkdir -p $O
export RMC_HOST_FRONTIER_GIB=245
lad() {  # module cfg tag
  t0=$(date +%s.%N)
  timeout -k 10 300 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module $1 -config configs/$2.cfg > $O/ladder_$3_auto.txt 2>&1
  rc=$?
  echo "$3 rc=$rc wall $(python3 -c "import time; print(round(time.time() - $t0, 2))")"
  grep -E "moved|host frontier:" $O/ladder_$3_auto.txt | cut -c1-200
  tail -1 $O/ladder_$3_auto.txt | cut -c1-200
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && exit 1
  return 0
}
lad FlexibleRaft FlexibleRaft FlexibleRaft
lad RaftFsync RaftFsync_n3v2e2r1 RaftFsync_n3v2e2r1
lad KRaft KRaft_n3v3e2 KRaft_n3v3e2
