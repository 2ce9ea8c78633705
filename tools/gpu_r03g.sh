#!/bin/bash
# debug: the fsync_n3v1e2r1 ladder prefix on two builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03g
mkdir -p $O
for b in build_pool build; do
timeout -k 10 120 python -u - $b > $O/run_$b.txt 2>&1 <<'PY'
import json, os, sys
sys.path.insert(0, "raft-tlaplus_amd")
import raftmc
raftmc.LIB_PATH = os.path.join("raft-tlaplus_amd", sys.argv[1], "librmc.so")
g = json.load(open("tests/golden/ladders.json"))["fsync_n3v1e2r1_rung"]
m = raftmc.Model(module=g["module"], cfg_path=g["cfg_path"])
for chunk in (0, 100000):
    r = m.check(max_depth=g["depth"], chunk_parents=chunk)
    print(sys.argv[1], chunk, {k: r[k] for k in ("status", "depth", "distinct", "generated", "message")}, r["levels"] == g["levels"], flush=True)
PY
echo "$b rc=$?"; cat $O/run_$b.txt | cut -c1-300
done
