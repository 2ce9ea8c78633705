#!/bin/bash
# r05e, on the default build (one tile per k_expand block): the logical-shard
# A/B of the generator-side tile dedup, fresh-process CLI checks of the bench
# workload on an idle GPU (each after a pause, so the driver has cleared the
# HBM the previous process freed), the config-5 rung RaftFsync_n3v1e2r2
# exhausted single-GPU and on 4 logical shards with host frontiers, then the
# profile set (bench line, kernel-trace stats, PMC passes: tools/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
O=$R/gpurun_out/r05e
mkdir -p $O
for w in 8 2; do
  for d in 1 0 1 0; do
    RMC_SHARD_DEDUP=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --logical-shards $w --steps 2 > $O/bench_logical${w}_dedup$d.json 2> $O/bench_logical${w}_dedup$d.err; rc=$?
    echo "logical $w dedup=$d rc=$rc $(python -c "import json; d=json.load(open('$O/bench_logical${w}_dedup$d.json')); print(d['ms_per_step'], d['result']['distinct'], d['result']['hidden_var_collisions'], d['kernel_ms'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
for i in 1 2 3; do
  sleep 45
  t0=$(date +%s.%N)
  timeout -k 10 120 $R/raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config $R/configs/Raft_n3v2e2.cfg > $O/cli_fresh_$i.txt 2>&1; rc=$?
  t1=$(date +%s.%N)
  echo "cli fresh #$i rc=$rc wall $(python -c "print(round($t1 - $t0, 3))") s, check $(python -c "import json; d=json.loads(open('$O/cli_fresh_$i.txt').read().strip().splitlines()[-1]); print(d['seconds'], d['distinct'])") $(grep -c 'rows widened' $O/cli_fresh_$i.txt) widenings"
  [ $rc -eq 0 ] || exit $rc
done
for a in "-hostfrontier -1" "-shards 4 -hostfrontier 1"; do
  tag=$(echo $a | tr -d ' -')
  timeout -k 10 200 $R/raft-tlaplus_amd/build/raftmc -deadlock -json -v $a -module RaftFsync -config $R/configs/RaftFsync_n3v1e2r2.cfg > $O/fsync_r2_$tag.txt 2>&1; rc=$?
  echo "RaftFsync_n3v1e2r2 $a rc=$rc $(tail -n 1 $O/fsync_r2_$tag.txt)"
  [ $rc -eq 0 ] || exit $rc
done
sleep 30
TAG=r05 timeout -k 10 900 bash tools/gpu_profile.sh > $O/profile.out 2>&1; rc=$?
echo "profile rc=$rc"; tail -n 25 $O/profile.out
exit $rc
