#!/bin/bash
# r03, fifth call: the whole -m gpu suite on the pooled-VMM build, a cold CLI
# after the driver has had time to clear the previous process's memory, bench,
# rocprof kernel stats, and the host-frontier ladders (auto switch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
CFG=configs/Raft_n3v2e2.cfg
for i in 1 2; do
  for b in build build_prev build_w8; do
    timeout -k 10 120 ./raft-tlaplus_amd/$b/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $CFG > $O/ab_${b}_$i.txt 2>&1 || { echo "$b failed"; exit 1; }
    echo "$b $(tail -1 $O/ab_${b}_$i.txt)"
  done
done
sleep 45
timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg > $O/cold_cli_after_sleep.txt 2>&1 || { echo "cold cli failed"; tail -5 $O/cold_cli_after_sleep.txt; exit 1; }
grep -E "setup|Finished|^\{" $O/cold_cli_after_sleep.txt
timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg > $O/cold_cli_right_after.txt 2>&1 || { echo "cold cli 2 failed"; exit 1; }
grep -E "Finished|^\{" $O/cold_cli_right_after.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $R/raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config $R/configs/Raft_n3v2e2.cfg > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/prof
head -5 $O/kernel_stats.csv | cut -c1-60
cd $R
export RMC_HOST_FRONTIER_GIB=240
for c in RaftFsync:RaftFsync_n3v2e2r1 KRaft:KRaft_n3v3e2 Raft:Raft_n3v2e3; do
  mod=${c%%:*}; cfg=${c##*:}
  timeout -k 10 500 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module $mod -config configs/$cfg.cfg > $O/ladder_${cfg}_hf.txt 2>&1; echo "$cfg rc=$?"
  grep -E "moved to host|Error|states generated|depth of|Finished" $O/ladder_${cfg}_hf.txt | cut -c1-200
done
