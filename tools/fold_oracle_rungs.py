"""Fold the C oracle's runs over the exhaustible BASELINE rungs
(tools/oracle_exhaust.py -> profiles/r04/oracle_<cfg>.json) into
tests/golden/exhausted.json.  TEST INFRASTRUCTURE ONLY (container).

For each rung the oracle's per-level (generated, new) pairs must equal the
GPU record's level for level (a prefix when the oracle run was truncated);
the record then carries them as `oracle` (levels, totals, hidden-variable
collisions, wall time, threads) and `oracle_levels` / `pinned_by` name the
C oracle.  Any difference aborts without writing.

    python tools/fold_oracle_rungs.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNS = {"fsync_n3v1e2r1_rung": "profiles/r04/oracle_RaftFsync_n3v1e2r1.json",
        "raft_n3v2e2_bench": "profiles/r04/oracle_Raft_n3v2e2.json",
        "fsync_n3v1e2r2_rung": "profiles/r05/oracle_RaftFsync_n3v1e2r2.json"}


def main():
    path = os.path.join(ROOT, "tests", "golden", "exhausted.json")
    ex = json.load(open(path))
    for name, rel in RUNS.items():
        p = os.path.join(ROOT, rel)
        if not os.path.exists(p):
            print("skip", name, "(no", rel + ")")
            continue
        o = json.load(open(p))
        g = ex[name]
        full = o["status"] == "ok"
        k = len(o["levels"]) if full else len(o["levels"]) - 1  # a truncated run's last level is partial
        if o["levels"][:k] != g["levels"][:k]:
            bad = next(i for i in range(k) if o["levels"][i] != g["levels"][i])
            raise SystemExit("%s: level %d differs: oracle %s, GPU %s" % (name, bad + 1, o["levels"][bad],
                                                                           g["levels"][bad]))
        if full and (o["generated"], o["distinct"], o["depth"], o["hidden_same_level"]) != (
                g["generated"], g["distinct"], g["depth"], g["hidden_var_collisions"]):
            raise SystemExit("%s: totals differ: oracle %s, GPU %s" % (
                name, (o["generated"], o["distinct"], o["depth"], o["hidden_same_level"]),
                (g["generated"], g["distinct"], g["depth"], g["hidden_var_collisions"])))
        g["oracle"] = dict(status=o["status"], levels=o["levels"][:k], generated=o["generated"],
                           distinct=o["distinct"], depth=o["depth"], hidden_same_level=o["hidden_same_level"],
                           seconds=o["seconds"], threads=o["threads"], source=rel)
        g["oracle_levels"] = k
        g["pinned_by"] = ("C oracle (oracle/cengine/rmc_oracle.cpp, exact canonical forms): %s; GPU rmc_check 64-bit "
                          "== 128-bit == 2 logical shards == host frontier" %
                          ("the whole rung, every level and total" if full else "the first %d levels" % k))
        print(name, "pinned:", g["pinned_by"])
    json.dump(ex, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    sys.exit(main())
