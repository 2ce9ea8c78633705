#!/bin/bash
# r04: kernel-trace stats of the 8-logical-shard bench (where the sharded protocol's time goes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt8 -o run --output-format csv -- python3 $R/bench.py --logical-shards 8 --no-cpu-baseline --steps 1 --warmup 1 > $O/kt8.log 2>&1 || { echo "kernel-trace failed"; tail -5 $O/kt8.log; exit 1; }
cp $(find $O/kt8 -name '*kernel_stats.csv' | head -1) $O/kernel_stats_logical8.csv
find $O -name '*kernel_trace.csv' -o -name '*agent_info.csv' | xargs rm -f
head -20 $O/kernel_stats_logical8.csv | cut -c1-200
