#!/bin/bash
# r04: chunk i's k_materialize on a second stream beside chunk i+1's k_expand.
# (1) bench with and without the overlap (same box, interleaved);
# (2) the whole -m gpu suite (minus the bench-rung host-frontier test, which
#     test_gpu_configs.py alone then runs with free HBM logged and polled).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04l}; mkdir -p $O
for v in 0 1 0 1; do
  RMC_NO_OVERLAP=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > $O/bench_noov$v.json 2> $O/bench_noov$v.err || { echo "bench $v failed"; tail -5 $O/bench_noov$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_noov$v.json')); print('no_overlap=$v', round(d['ms_per_step'],1), d['kernel_ms'], d['result']['distinct'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect "tests/test_gpu_configs.py::test_rung_host_frontier[raft_n3v2e2_bench]" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
RMC_TEST_MEMLOG=$O/memlog.txt RMC_TEST_MEMLOG_POLL=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_configs.log 2>&1; echo "configs rc=$?"
tail -3 $O/pytest_configs.log
cut -c1-160 $O/memlog.txt
