#!/bin/bash
# r03, fourth call: parity of the new k_materialize (lockstep row merge,
# invariants in place), A/B timing vs the r02-equivalent build, VMM release
# semantics, cold CLI with t_grow breakdown, bench, available counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_extras.py tests/test_gpu_n5.py tests/test_gpu_sharded_mp.py tests/test_gpu_sharded.py tests/test_gpu_flex_restart.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
CFG=configs/Raft_n3v2e2.cfg
run() {  # build tag
  timeout -k 10 120 ./raft-tlaplus_amd/$1/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $CFG > $O/$2.txt 2>&1 || { echo "$1 failed"; tail -3 $O/$2.txt; exit 1; }
  echo "$1 $(tail -1 $O/$2.txt)"
}
for i in 1 2; do
  for b in build build_r02 build_ml256; do run $b ${b}_$i; done
done
timeout -k 10 120 ./tools/probe/vmm_release_probe > $O/vmm_release_probe.txt 2>&1; echo "probe rc=$?"
cat $O/vmm_release_probe.txt
timeout -k 10 120 ./raft-tlaplus_amd/build/raftmc -deadlock -json -v -module Raft -config $CFG > $O/cold_cli.txt 2>&1 || { echo "cold cli failed"; tail -5 $O/cold_cli.txt; exit 1; }
grep -E "setup|grown|Finished|^\{" $O/cold_cli.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_avail.txt 2>&1; echo "list rc=$?"
