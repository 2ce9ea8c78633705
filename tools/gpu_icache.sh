#!/bin/bash
# Is k_expand bound by instruction fetch?  rocprofv3 counter list, then the
# SQC instruction-cache counters and SQ fetch/wait counters over one check of
# the bench cfg (separate --pmc passes, each under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/icache
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INSTS_[A-Z_0-9]*" $O/avail.txt | sort -u > $O/names.txt
CLI="$R/raft-tlaplus_amd/${B:-build}/raftmc -deadlock -json -hashslots 4294967296 -module Raft -config $R/configs/Raft_n3v2e2.cfg"
pass() {
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$tag -o run --output-format csv -- $CLI > $O/$tag.log 2>&1
  local rc=$?
  echo "pass $tag rc=$rc"
  if [ $rc -eq 0 ]; then
    python3 $R/tools/pmc_summary.py $O/$tag.json --pmc $(find $O/$tag -name '*counter_collection.csv' | head -1) > /dev/null
    python3 -c "
import json; d=json.load(open('$O/$tag.json'))
for k,v in d['kernels'].items():
    if k.startswith('rmc::k_'): print('$tag', k, {a:round(b) for a,b in v.items() if a.endswith('per_dispatch')})"
    rm -rf $O/$tag
  fi
  return $rc
}
for c in $(cat $O/names.txt | tr '\n' ' '); do echo -n "$c "; done; echo
pass ic1 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
rc=$?; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
pass ic2 SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY
rc=$?; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
exit 0
