#!/bin/bash
# r06 (session 2) closing pass on the final build (phase-B wave sync, no REF load):
# smoke, the profile (bench line, kernel trace, PMC passes), then the
# sharded protocol on 8 and 2 logical shards of the one GPU (k_insert_recv,
# k_mark_recv, k_mark_gen, k_bucket, k_owner_count with batched loads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r/pytest_r.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" gpurun_out/r/pytest_r.log | head -20; tail -30 gpurun_out/r/pytest_r.log; exit 1; }
tail -2 gpurun_out/r/pytest_r.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r/smoke_r.log 2>&1 || { echo smoke failed; cat gpurun_out/r/smoke_r.log; exit 1; }
cat gpurun_out/r/smoke_r.log
TAG=r06s5 bash tools/gpu_profile.sh || { echo "profile failed"; exit 1; }
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r/bench_logical_$W.json 2> gpurun_out/r/bench_logical_$W.err \
    || { echo "logical $W failed"; tail -5 gpurun_out/r/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r/bench_logical_$W.json')); print('logical $W', d['ms_per_step'], d['result']['distinct'], d['result'].get('hidden_var_collisions'), d.get('kernel_ms'))"
done
SHARDS=8 LIMIT=200 bash tools/gpu_shards_prof.sh && python3 tools/rocpd_summary.py gpurun_out/shprof_8/run_results.db > gpurun_out/r/kernels_logical8_cli.txt && head -12 gpurun_out/r/kernels_logical8_cli.txt
