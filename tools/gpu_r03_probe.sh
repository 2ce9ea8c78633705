#!/bin/bash
# r03: read-only probing in fpset_insert.  Insert-protocol counts (RMC_FPSTATS
# builds, r02 protocol vs new), CLI timing A/B, WRITE_SIZE per build, then the
# parity + TLC-order GPU tests on the new build.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r03_probe
mkdir -p $O
CFG=${CFG:-Raft_n3v2e2}
run() {  # build tag
  timeout -k 10 120 ./raft-tlaplus_amd/$1/raftmc -deadlock -json -v -hashslots 4294967296 -module Raft -config configs/$CFG.cfg > $O/$2.txt 2>&1 || { echo "$1 failed"; tail -3 $O/$2.txt; exit 1; }
  echo "$1 $(grep -h 'fingerprint-set inserts' $O/$2.txt) $(tail -1 $O/$2.txt)"
}
run build_lstats lstats
run build_stats stats
for i in 1 2; do
  run build_legacy legacy_$i
  run build new_$i
done
cd /tmp && export TMPDIR=/tmp
for v in build_legacy build; do
  P=$O/pmc_$v
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $P -o run --output-format csv -- $R/raft-tlaplus_amd/$v/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $R/configs/$CFG.cfg > $P.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 $R/tools/pmc_summary.py $P.json --pmc $(find $P -name '*counter_collection.csv' | head -1) > /dev/null
  python3 -c "
import json; d=json.load(open('$P.json'))
for k,v in d['kernels'].items():
    if k.startswith('rmc::k_'): print('$v WRITE_SIZE', k, '%.4g MB/dispatch' % (v['WRITE_SIZE_per_dispatch']*1024/1e6))"
  rm -rf $P
done
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
exit $rc
