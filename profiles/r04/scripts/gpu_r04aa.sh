#!/bin/bash
# r04: the bench workload's mean row bytes up to the last message
# (build_rowstats, -DRMC_ROWSTATS, CLI -v), then the simulation / parity /
# checkpoint suites on build after DevStatus grew a field.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${TAG:-r04aa}; mkdir -p $O
timeout -k 10 120 ./raft-tlaplus_amd/build_rowstats/raftmc -deadlock -json -v -module Raft -config configs/Raft_n3v2e2.cfg > $O/rowstats.txt 2>&1 || { echo "rowstats failed"; tail -3 $O/rowstats.txt; exit 1; }
grep -E "rows:|expand_ms" $O/rowstats.txt | cut -c1-300
timeout -k 10 600 python -u -m pytest tests/test_gpu_simulate.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_trace.py tests/test_gpu_extras.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
