#!/bin/bash
# r04: per-shard host frontier + level-boundary auto switch + per-shard HBM accounting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r04g}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_host_frontier.py tests/test_gpu_configs.py tests/test_gpu_sharded_mp.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=8 > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
