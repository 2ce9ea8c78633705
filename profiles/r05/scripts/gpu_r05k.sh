#!/bin/bash
# r05k: the GPU record of config 5's rung RaftFsync_n3v1e2r2 (64-bit == 128-bit
# == 2 logical shards == host frontier) for tests/golden/exhausted.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05k
timeout -k 10 600 python -u tools/make_exhausted_record.py gpurun_out/r05k/exhausted_r2.json --only=fsync_n3v1e2r2_rung
