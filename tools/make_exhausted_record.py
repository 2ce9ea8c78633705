"""Record the exhaustive GPU results of the exhaustible BASELINE rungs
(tests/golden/exhausted.json) -- run on the GPU box:

    python tools/make_exhausted_record.py gpurun_out/exhausted.json [--only=name,...]

These state spaces (10^8-10^9 distinct states) are beyond the oracles'
reach; each record is written only if the 64-bit check, the 128-bit check,
2 logical shards and the host-memory frontier all agree on generated,
distinct, depth, every per-level pair and the hidden-variable collisions, and
if its first levels equal both oracles' (tests/golden/ladders.json).  The
tests then pin these counts (regression) and re-check the agreement."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-tlaplus_amd"))
import raftmc  # noqa: E402

RUNGS = [("raft_n3v2e2_bench", "Raft", "configs/Raft_n3v2e2.cfg"),
         ("fsync_n3v1e2r1_rung", "RaftFsync", "configs/RaftFsync_n3v1e2r1.cfg"),
         # r05: config 5's largest rung one node holds; no ladder
         # prefix -- the C oracle's full run pins every level (fold_oracle_rungs.py)
         ("fsync_n3v1e2r2_rung", "RaftFsync", "configs/RaftFsync_n3v1e2r2.cfg")]
KEYS = ("generated", "distinct", "depth", "status", "levels", "hidden_var_collisions")


def main():
    lad = json.load(open(os.path.join(ROOT, "tests", "golden", "ladders.json")))
    out = {}
    only = [a.split("=", 1)[1].split(",") for a in sys.argv[2:] if a.startswith("--only=")]
    for name, module, cfg in RUNGS:
        if only and name not in only[0]:
            continue
        m = raftmc.Model(module=module, cfg_path=os.path.join(ROOT, cfg))
        runs = {}
        for tag, fn in (("fp64", m.check), ("fp128", lambda: m.check(fp_bits=128)),
                        ("shards2", lambda: m.check_logical(2)), ("host_frontier", lambda: m.check(host_frontier=1))):
            raftmc.release_device_memory()  # each mode starts from an empty device
            runs[tag] = fn()
        base = {k: runs["fp64"][k] for k in KEYS}
        for tag, r in runs.items():
            got = {k: r[k] for k in KEYS}
            if got != base:
                raise SystemExit("%s: %s disagrees with fp64: %s" % (name, tag, {k: (got[k], base[k]) for k in KEYS
                                                                               if got[k] != base[k]}))
        k = 0
        if name in lad:
            g = lad[name]
            k = len(g["levels"]) - 1  # the oracles' last (truncated) level is partial
            if base["levels"][:k] != g["levels"][:k]:
                raise SystemExit("%s: first %d levels differ from the oracles'" % (name, k))
        out[name] = dict(module=module, cfg_path=cfg, oracle_levels=k,
                         pinned_by="GPU rmc_check; 64-bit == 128-bit == 2 logical shards == host frontier" +
                                   ("; first %d levels == both oracles (ladders.json)" % k if k else ""), **base)
        print(name, base["generated"], base["distinct"], base["depth"], base["hidden_var_collisions"],
              {t: round(r["seconds"], 3) for t, r in runs.items()}, flush=True)
    with open(sys.argv[1], "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
