#!/bin/bash
# r05h: bench.py right after a ~150 GB process (the driver's order: pytest / smoke, then the
# bench), with the bench's wait for freed HBM before its warm-up check
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
O=$R/gpurun_out/r05h
mkdir -p $O
timeout -k 10 120 $R/raft-tlaplus_amd/build/raftmc -deadlock -json -module Raft -config $R/configs/Raft_n3v2e2.cfg > $O/cli_before.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['result']; print(d['ms_per_step'], r['first_check_s'], r['hbm_wait_s'], r['hbm_free_frac'])"
