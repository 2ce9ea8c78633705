#!/bin/bash
# r05: the persistent k_expand (LDS-DMA prefetch of the block's next tile) --
# the whole -m gpu suite on it, the bench line A/B against the one-tile-per-
# block build (build_np, -DRMC_EXPAND_PERSIST=0), the kernel-trace summary of
# the bench, a fresh-process CLI check of the bench workload, and host-frontier
# ladders of the candidate config-5 rungs (last: they may run into their limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
O=$R/gpurun_out/r05d
mkdir -p $O
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 3 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for b in build build_np; do
    RAFTMC_BUILD=$b timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_${b}_$i.json 2> $O/bench_${b}_$i.err; rc=$?
    echo "$b #$i rc=$rc $(python -c "import json; d=json.load(open('$O/bench_${b}_$i.json')); print(d['ms_per_step'], d['kernel_ms'], d['result']['first_check_s'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
# a fresh process per check (what a user's first raftmc run costs)
for b in build build_np; do
  for i in 1 2; do
    t0=$(date +%s.%N)
    timeout -k 10 120 $R/raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config $R/configs/Raft_n3v2e2.cfg > $O/cli_${b}_$i.json 2> $O/cli_${b}_$i.err; rc=$?
    t1=$(date +%s.%N)
    echo "cli $b #$i rc=$rc wall $(python -c "print(round($t1 - $t0, 3))") s, check $(python -c "import json; d=json.loads(open('$O/cli_${b}_$i.json').read().strip().splitlines()[-1]); print(d['seconds'], d['distinct'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
# logical shards: the generator-side tile dedup (default) against none
for w in 8 2; do
  for d in 1 0; do
    RMC_SHARD_DEDUP=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --logical-shards $w --steps 2 > $O/bench_logical${w}_dedup$d.json 2> $O/bench_logical${w}_dedup$d.err; rc=$?
    echo "logical $w dedup=$d rc=$rc $(python -c "import json; d=json.load(open('$O/bench_logical${w}_dedup$d.json')); print(d['ms_per_step'], d['result']['distinct'], d['result']['hidden_var_collisions'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/kt.log 2>&1 || { echo "kernel-trace failed"; exit 1; }
cp $(find $O/kt -name '*kernel_stats.csv' | head -n 1) $O/kernel_stats.csv
find $O/kt -name '*kernel_trace.csv' -o -name '*agent_info.csv' | xargs rm -f
head -n 6 $O/kernel_stats.csv
cd $R
for mc in $RUNGS; do  # Module:cfg
  mod=${mc%%:*}; cfg=${mc#*:}
  timeout -k 10 ${RUNG_LIMIT:-150} ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -hostfrontier 1 -module $mod -config configs/$cfg.cfg > $O/ladder_$cfg.txt 2>&1; rc=$?
  echo "$cfg rc=$rc"; tail -n 2 $O/ladder_$cfg.txt
  [ $rc -eq 0 ] || [ $rc -eq 12 ] || [ $rc -eq 13 ] || exit $rc
done
exit 0
