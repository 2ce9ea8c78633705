#!/bin/bash
# r03, second call: exhausted-rung records, the new GPU tests (host frontier,
# configs 2/5, checkpoint, simulation replay), cold CLI timing, bench + kernel
# stats, and config 2 (Raft_n3v2e3) with the host frontier.  Stops at the
# first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03b
mkdir -p $O
free -g > $O/host_mem.txt; df -h /tmp $R >> $O/host_mem.txt; nproc >> $O/host_mem.txt
timeout -k 10 300 python -u tools/make_exhausted_record.py $O/exhausted.json > $O/exhausted.log 2>&1 || { echo "record failed"; tail -5 $O/exhausted.log; exit 1; }
cat $O/exhausted.log
cp $O/exhausted.json tests/golden/exhausted.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_frontier.py tests/test_gpu_configs.py tests/test_gpu_checkpoint.py tests/test_gpu_simulate.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg > $O/cold_cli.txt 2>&1 || { echo "cold cli failed"; tail -5 $O/cold_cli.txt; exit 1; }
grep -E "setup|grown|Finished" $O/cold_cli.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $R/raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config $R/configs/Raft_n3v2e2.cfg > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/prof
head -8 $O/kernel_stats.csv
cd $R
timeout -k 10 400 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e3.cfg > $O/cfg2_hostfrontier.txt 2>&1; echo "cfg2 rc=$?"
tail -12 $O/cfg2_hostfrontier.txt | cut -c1-400
