#!/bin/bash
# One gpurun call: the bench line, the rocprofv3 kernel-trace summary of the
# same bench command, and separate --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ
# counters) over one check of the same workload through the CLI.  Every GPU
# step has its own time limit; the script stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-r02}
WL=${WL:-raft_n3v2e2}
CFG=${CFG:-Raft_n3v2e2}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
set -o pipefail
timeout -k 10 420 python -u bench.py --workload $WL $BENCH_ARGS > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --workload $WL --no-cpu-baseline --steps 2 --warmup 1 > $O/kt.log 2>&1 || { echo "kernel-trace failed"; exit 1; }
CLI="$R/raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config $R/configs/$CFG.cfg"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc1 -o run --output-format csv -- $CLI > $O/pmc1.log 2>&1 || { echo "pmc1 failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc2 -o run --output-format csv -- $CLI > $O/pmc2.log 2>&1 || { echo "pmc2 failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc3 -o run --output-format csv -- $CLI > $O/pmc3.log 2>&1 || { echo "pmc3 failed"; exit 1; }
# counter calibration for random (non-streaming) accesses: known access counts
CAL="$R/raft-tlaplus_amd/build/fpset_bench -calib -slots_log2 30 -batch 67108864"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal1 -o run --output-format csv -- $CAL > $O/cal1.log 2>&1 || { echo "cal1 failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/cal2 -o run --output-format csv -- $CAL > $O/cal2.log 2>&1 || { echo "cal2 failed"; exit 1; }
cd $R
python3 tools/pmc_summary.py $O/calib.json --pmc $(find $O/cal1 -name '*counter_collection.csv' | head -1) \
  --pmc $(find $O/cal2 -name '*counter_collection.csv' | head -1) > /dev/null 2>&1
grep calib $O/cal1.log
python3 tools/pmc_summary.py $O/summary.json --workload $WL --stats $(ls $O/kt/*kernel_stats.csv | head -1) \
  --pmc $(find $O/pmc1 -name '*counter_collection.csv' | head -1) --pmc $(find $O/pmc2 -name '*counter_collection.csv' | head -1) \
  --pmc $(find $O/pmc3 -name '*counter_collection.csv' | head -1) > $O/summary.txt 2>&1
echo "summary rc=$?"
cat $O/summary.txt
# keep summaries only: raw per-dispatch CSVs exceed gpurun's 64 MiB copy-back limit
cp $(find $O/kt -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
find $O -name '*counter_collection.csv' -o -name '*kernel_trace.csv' -o -name '*agent_info.csv' | xargs rm -f
du -sh $O
