#!/bin/bash
# r06 fourth GPU pass: where a first check's table growth goes.  The bench
# warm-up on a fresh box, then a CLI check of the same workload (~150 GB of
# HBM allocated and freed), then the bench warm-up again: rmc_check_phases
# splits table_growth into allocate (hipMalloc of each doubled set) / fill /
# rehash.  Then the handler GPU tests (HandleAppendEntriesResponse cases) and
# the phases test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/d
timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/d/bench_fresh.json 2> gpurun_out/d/bench_fresh.err \
  || { echo "bench 1 failed"; tail -5 gpurun_out/d/bench_fresh.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/d/bench_fresh.json')); print('fresh', d['result']['first_check_phases'])"
timeout -k 10 200 raft-tlaplus_amd/build/raftmc -deadlock -v -json -module Raft -config configs/Raft_n3v2e2.cfg > gpurun_out/d/cli.txt 2>&1 \
  || { echo "cli failed"; tail -5 gpurun_out/d/cli.txt; exit 1; }
grep -E "grown|Finished" gpurun_out/d/cli.txt
timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/d/bench_after.json 2> gpurun_out/d/bench_after.err \
  || { echo "bench 2 failed"; tail -5 gpurun_out/d/bench_after.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/d/bench_after.json')); print('after', d['result']['first_check_phases'])"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_handlers.py \
  "tests/test_gpu_host_frontier.py::test_first_check_phases_add_up" > gpurun_out/d/pytest_d.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/d/pytest_d.log | head; tail -20 gpurun_out/d/pytest_d.log; exit 1; }
tail -1 gpurun_out/d/pytest_d.log
