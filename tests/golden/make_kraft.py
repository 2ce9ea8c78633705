"""Generate tests/golden/kraft.json: KRaft (pull-raft/KRaft.tla).

Run in the build container:  python tests/golden/make_kraft.py

Each case is computed by the literal Python oracle (oracle/pyoracle/kraft.py)
AND the independent C++ oracle (oracle/cengine/kraft_oracle.cpp, `make -C
oracle`) under TLC -workers 1 semantics, and written only if they agree on
generated / distinct / depth, every per-level count, hidden-variable
collisions and the per-action successor counts; the violated invariant and
trace length of the unsafe ones (KRaft with MaxRestarts >= 1 reaches
IllegalState) come from the Python oracle.  The shipped cfg (pull-raft/
KRaft.cfg: N=3, V=1, E=2) is added level-truncated for both oracles
(--shipped-levels, default 30000 states) and, with --shipped-full, exhausted by
the C++ oracle alone (about 20 minutes).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle.pyoracle import make_spec  # noqa: E402
from oracle.pyoracle.cfg import parse_cfg  # noqa: E402
from oracle.pyoracle.tlc import bfs  # noqa: E402
from cfgs import KRAFT, kraft_cfg_text  # noqa: E402
from oracle import run_c  # noqa: E402


def record(txt, max_states=None):
    r = bfs(make_spec("KRaft", parse_cfg(txt)), max_states=max_states)
    cfg = parse_cfg(txt)
    c = run_c.run_kraft(cfg["constants"], cfg["invariants"], max_states=max_states or 0)
    if (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"], c["hidden_same_level"],
            c["action_counts"]) != (r.generated, r.distinct, r.depth, r.status, [list(x) for x in r.levels],
                                    r.hidden_same_level, r.action_counts):
        raise SystemExit("KRaft oracles disagree:\n%s" % txt)
    out = dict(module="KRaft", cfg=txt, generated=r.generated, distinct=r.distinct, depth=r.depth,
               status=r.status, levels=[list(x) for x in r.levels], max_msgs=r.max_msgs,
               hidden_same_level=r.hidden_same_level, action_counts=r.action_counts, pinned_by="pyoracle==coracle")
    if r.status == "violation":
        out["violated"] = r.violated
        out["trace_len"] = len(r.trace)
    if max_states:
        out["max_states"] = max_states
    return out


def main():
    out = {}
    for name, kw in KRAFT:
        out[name] = record(kraft_cfg_text(**kw))
        g = out[name]
        print(name, g["generated"], g["distinct"], g["depth"], g["status"], g.get("violated"), flush=True)
    n = 30000
    for a in sys.argv[1:]:
        if a.startswith("--shipped-levels="):
            n = int(a.split("=", 1)[1])
    out["KRaft_cfg_prefix"] = record(kraft_cfg_text(n=3, v=1, E=2, R=0), max_states=n)
    g = out["KRaft_cfg_prefix"]
    print("KRaft_cfg_prefix", g["generated"], g["distinct"], g["depth"], g["status"], flush=True)
    if "--shipped-full" in sys.argv:
        txt = kraft_cfg_text(n=3, v=1, E=2, R=0)
        cfg = parse_cfg(txt)
        c = run_c.run_kraft(cfg["constants"], cfg["invariants"])
        out["KRaft_cfg"] = dict(module="KRaft", cfg=txt, generated=c["generated"], distinct=c["distinct"],
                                depth=c["depth"], status=c["status"], levels=c["levels"], max_msgs=c["max_msgs"],
                                hidden_same_level=c["hidden_same_level"], action_counts=c["action_counts"],
                                pinned_by="coracle (first %d levels pyoracle==coracle)" % len(g["levels"]))
        print("KRaft_cfg", c["generated"], c["distinct"], c["depth"], c["status"], flush=True)
    with open(os.path.join(HERE, "kraft.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
