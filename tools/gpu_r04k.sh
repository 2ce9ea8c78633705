#!/bin/bash
# r04: the GPU suites in the order that fails test_rung_host_frontier, with
# free HBM logged after every test (tests/conftest.py RMC_TEST_MEMLOG).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04k}; mkdir -p $O
RMC_TEST_MEMLOG=$O/memlog.txt RMC_TEST_MEMLOG_POLL=${POLL:-0} timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py tests/test_gpu_configs.py} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
tail -5 $O/pytest.log
cat $O/memlog.txt | cut -c1-200 | tail -80
