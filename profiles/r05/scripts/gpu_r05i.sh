#!/bin/bash
# r05i: the CPU engine (raftmc -cpu, 16 worker threads: the box's CPU share)
# over the WHOLE bench workload on the GPU box's host -- the same-host
# time-to-exhaust beside the GPU's (bench.py's cpu_baseline samples a prefix)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
R=$PWD
O=$R/gpurun_out/r05i
mkdir -p $O
lscpu | grep -E "Model name|^CPU\(s\)" > $O/host.txt
t0=$(date +%s.%N)
timeout -k 10 1080 $R/raft-tlaplus_amd/build/raftmc -cpu -workers 16 -deadlock -json -v -module Raft -config $R/configs/Raft_n3v2e2.cfg > $O/cpu_full_raft_n3v2e2.txt 2>&1; rc=$?
t1=$(date +%s.%N)
echo "cpu engine rc=$rc wall $(python -c "print(round($t1 - $t0, 1))") s $(tail -n 1 $O/cpu_full_raft_n3v2e2.txt)"
exit $rc
