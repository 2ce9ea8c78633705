#!/bin/bash
# r06 (session 2): k_mark_gen as a wave per tile (k_mark_gen_tiles) -- the
# whole -m gpu suite on this build, smoke, the bench line, then the sharded
# protocol on 8 and 2 logical shards and a kernel trace of the 8-shard CLI
# check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/n
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/n/pytest_n.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" gpurun_out/n/pytest_n.log | head -20; tail -30 gpurun_out/n/pytest_n.log; exit 1; }
tail -2 gpurun_out/n/pytest_n.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/n/smoke_n.log 2>&1 || { echo smoke failed; cat gpurun_out/n/smoke_n.log; exit 1; }
cat gpurun_out/n/smoke_n.log
timeout -k 10 300 python bench.py > gpurun_out/n/bench_n.json 2> gpurun_out/n/bench_n.err || { echo "bench failed"; tail -20 gpurun_out/n/bench_n.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/n/bench_n.json')); print('bench', d['ms_per_step'], d['value'], d['kernel_ms'])"
for W in 8 2; do
  timeout -k 10 300 python -u bench.py --logical-shards $W --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/n/bench_logical_$W.json 2> gpurun_out/n/bench_logical_$W.err \
    || { echo "logical $W failed"; tail -5 gpurun_out/n/bench_logical_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/n/bench_logical_$W.json')); print('logical $W', d['ms_per_step'], d['result']['distinct'], d['result'].get('hidden_var_collisions'), d.get('kernel_ms'))"
done
SHARDS=8 LIMIT=200 bash tools/gpu_shards_prof.sh && python3 tools/rocpd_summary.py gpurun_out/shprof_8/run_results.db > gpurun_out/n/kernels_logical8_cli.txt
head -12 gpurun_out/n/kernels_logical8_cli.txt
