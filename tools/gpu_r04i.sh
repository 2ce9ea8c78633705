#!/bin/bash
# r04: (1) the rung host-frontier tests' suite order with device free memory
# printed after every check (tools/hf_dbg.py); (2) the bench workload on 8
# and 2 logical shards (alignment-aware batched copies) + kernel stats at W=8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r04i; mkdir -p $O
timeout -k 10 400 python -u tools/hf_dbg.py > $O/hf_dbg.txt 2>&1; echo "hf_dbg rc=$?"; grep -vE "^\[rmc\] depth ([0-9]|[1-3][0-9]):" $O/hf_dbg.txt | tail -30
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --no-cpu-baseline --steps 2 > $O/bench_logical_$W.json 2> $O/bench_logical_$W.err || { echo "bench W=$W failed"; tail -5 $O/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_logical_$W.json')); print($W, d['ms_per_step'], d['kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt8 -o run --output-format csv -- python3 $R/bench.py --logical-shards 8 --no-cpu-baseline --steps 1 --warmup 1 > $O/kt8.log 2>&1 || { echo "kernel-trace failed"; tail -5 $O/kt8.log; exit 1; }
cp $(find $O/kt8 -name '*kernel_stats.csv' | head -1) $O/kernel_stats_logical8.csv
find $O/kt8 -name '*.csv' | xargs rm -f
head -12 $O/kernel_stats_logical8.csv | cut -c1-160
