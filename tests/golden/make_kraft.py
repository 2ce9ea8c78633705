"""Generate tests/golden/kraft.json: KRaft (pull-raft/KRaft.tla).

Run in the build container:  python tests/golden/make_kraft.py

Each case is the literal Python oracle (oracle/pyoracle/kraft.py) under TLC
-workers 1 semantics: generated / distinct / depth, every per-level count,
hidden-variable collisions, the violated invariant and trace length of the
unsafe ones (KRaft with MaxRestarts >= 1 reaches IllegalState).  Only one
restatement pins these (the C oracle does not lower KRaft): parity is pinned
by that oracle alone, and the GPU lowering (rmc_spec.h kr_*) is written
independently of it.  The shipped cfg (pull-raft/KRaft.cfg: N=3, V=1, E=2) is
added level-truncated (--shipped-levels, default 30000 states).
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


def record(txt, max_states=None):
    r = bfs(make_spec("KRaft", parse_cfg(txt)), max_states=max_states)
    out = dict(module="KRaft", cfg=txt, generated=r.generated, distinct=r.distinct, depth=r.depth,
               status=r.status, levels=[list(x) for x in r.levels], max_msgs=r.max_msgs,
               hidden_same_level=r.hidden_same_level, action_counts=r.action_counts, pinned_by="pyoracle")
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
    with open(os.path.join(HERE, "kraft.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
