#!/usr/bin/env python3
"""k_expand phase costs on a real BFS level (RMC_DIAG builds of librmc):
   profile_expand.py BUILD_DIR LEVEL [CFG]
Checks the cfg up to LEVEL, then times LEVEL's first chunk of k_expand stopped
after each phase (4 staging, 3 + bindings, 2 + successor deltas, 1 + fingerprints /
tile dedup, 0 the real launch with inserts); one JSON line."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-tlaplus_amd"))
import raftmc  # noqa: E402

build, level = sys.argv[1], int(sys.argv[2])
cfg = sys.argv[3] if len(sys.argv) > 3 else "configs/Raft_n3v2e2.cfg"
raftmc.LIB_PATH = os.path.join(ROOT, "raft-tlaplus_amd", build, "librmc.so")
m = raftmc.Model(module="Raft", cfg_path=os.path.join(ROOT, cfg))
prof = m.selftest_profile_expand(level, hash_slots=1 << 32)
by = {}
for d, ms in prof:
    by.setdefault(d, []).append(ms)
out = {"build": build, "level": level, "cfg": cfg,
       "ms": {str(d): round(statistics.median(v), 4) for d, v in sorted(by.items())}}
names = {4: "staging", 3: "bindings", 2: "deltas", 1: "fingerprints", 0: "inserts"}
prev = 0.0
out["phase_ms"] = {}
for d in (4, 3, 2, 1, 0):
    if d in by:
        t = statistics.median(by[d])
        out["phase_ms"][names[d]] = round(t - prev, 4)
        prev = t
print(json.dumps(out), flush=True)
