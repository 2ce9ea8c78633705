#!/bin/bash
# r06 (session 2): records per owner thread in k_insert_recv / k_mark_recv
# (RMC_RECV_U = 2 / 4 / 8) after their loads were batched; bench.py on 8
# logical shards (steady-state checks), interleaved, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
for round in 1 2; do
  for b in build_u2 build_u4 build_u8; do
    RAFTMC_BUILD=$b timeout -k 10 300 python -u bench.py --logical-shards 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s/ab_${b}_${round}.json 2> gpurun_out/s/ab_${b}_${round}.err \
      || { echo "ab $b failed"; tail -5 gpurun_out/s/ab_${b}_${round}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/s/ab_${b}_${round}.json')); print('$b round $round', d['ms_per_step'], d['result']['distinct'], d['result'].get('hidden_var_collisions'))"
  done
done | tee gpurun_out/s/ab_recv_u.txt || { echo "ab loop failed"; exit 1; }
