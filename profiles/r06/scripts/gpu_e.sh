#!/bin/bash
# r06: (1) where a first check's table growth goes (bench warm-up on a fresh
# box, a CLI check of the same workload that allocates and frees ~150 GB,
# the bench warm-up again; rmc_check_phases splits table_growth into
# allocate / fill / rehash); (2) k_materialize occupancy A/B: the default
# build (512-entry winner list, 95 VGPRs: LDS allows 9 blocks per CU), a
# 128- and a 256-entry list, and a 128-entry list with 6 waves per SIMD
# forced; CLI, interleaved, two rounds; (3) the handler GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e
timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/e/bench_fresh.json 2> gpurun_out/e/bench_fresh.err \
  || { echo "bench 1 failed"; tail -5 gpurun_out/e/bench_fresh.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/e/bench_fresh.json')); print('fresh', d['result']['first_check_phases'])"
timeout -k 10 200 raft-tlaplus_amd/build/raftmc -deadlock -v -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/e/cli.txt 2>&1 \
  || { echo "cli failed"; tail -5 gpurun_out/e/cli.txt; exit 1; }
grep -E "grown|Finished" gpurun_out/e/cli.txt
timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/e/bench_after.json 2> gpurun_out/e/bench_after.err \
  || { echo "bench 2 failed"; tail -5 gpurun_out/e/bench_after.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/e/bench_after.json')); print('after', d['result']['first_check_phases'])"
for round in 1 2; do
  for b in build build_ml128 build_ml256 build_ml128w6; do
    timeout -k 10 120 raft-tlaplus_amd/$b/raftmc -deadlock -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/e/ab_${b}_${round}.txt 2>&1 \
      || { echo "ab $b failed"; tail -5 gpurun_out/e/ab_${b}_${round}.txt; exit 1; }
    echo "$b round $round $(tail -1 gpurun_out/e/ab_${b}_${round}.txt)"
  done
done | tee gpurun_out/e/ab_materialize.txt || { echo "ab loop failed"; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_handlers.py \
  "tests/test_gpu_host_frontier.py::test_first_check_phases_add_up" > gpurun_out/e/pytest_e.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/e/pytest_e.log | head; tail -20 gpurun_out/e/pytest_e.log; exit 1; }
tail -1 gpurun_out/e/pytest_e.log
