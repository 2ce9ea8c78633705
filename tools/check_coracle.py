"""Re-run the C oracle on every committed fixture and compare.  TEST INFRASTRUCTURE ONLY.

Used after a change to oracle/cengine/rmc_oracle.cpp's engine (not its
restatement of the specs): every fixture's generated / distinct / depth /
per-level counts / hidden-variable collisions / status / violated invariant /
trace length must come out unchanged, at 1 and 8 threads, and the TLC-order
fixtures' --reverse-order counts too.

    python tools/check_coracle.py [--threads 8] [--skip-large]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import run_c  # noqa: E402
from oracle.pyoracle.cfg import parse_cfg  # noqa: E402

FILES = ["small.json", "medium.json", "order.json", "n5.json", "shipped.json", "variant2.json", "extras.json",
         "flex_restart.json", "ladders.json", "unsafe.json"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--skip-large", action="store_true", help="skip fixtures above 2e6 distinct")
    a = ap.parse_args()
    bad = 0
    for fn in FILES:
        p = os.path.join(ROOT, "tests", "golden", fn)
        if not os.path.exists(p):
            continue
        for name, g in sorted(json.load(open(p)).items()):
            if not isinstance(g, dict) or g.get("module") not in ("Raft", "FlexibleRaft", "RaftFsync", "PullRaft",
                                                                    "PullRaftVariant2"):
                continue
            if a.skip_large and g.get("distinct", 0) > 2_000_000:
                continue
            txt = g.get("cfg") or open(os.path.join(ROOT, g["cfg_path"])).read()
            cfg = parse_cfg(txt)
            extra = []
            if g.get("max_distinct"):
                extra += ["--max-distinct", str(g["max_distinct"])]
            want_trace = "trace_len" in g
            if want_trace:
                extra += ["--trace"]
            t0 = time.time()
            c = run_c.run(g["module"], cfg["constants"], cfg["invariants"], threads=a.threads, extra=extra)
            diffs = []
            for k in ("generated", "distinct", "depth", "status", "levels", "hidden_same_level", "violated",
                      "hidden_cross_level", "max_msgs"):
                if k in g and g[k] != c.get(k):
                    diffs.append(k)
            if want_trace and g["trace_len"] != len(c.get("trace", [])):
                diffs.append("trace_len")
            if "reverse_order" in g:
                rv = run_c.run(g["module"], cfg["constants"], cfg["invariants"], threads=1,
                               extra=extra + ["--reverse-order"])
                if (rv["generated"], rv["distinct"]) != (g["reverse_order"]["generated"],
                                                         g["reverse_order"]["distinct"]):
                    diffs.append("reverse_order")
            print("%-14s %-36s %s %.1fs" % (fn, name, "OK" if not diffs else "DIFF " + ",".join(diffs),
                                            time.time() - t0), flush=True)
            bad += bool(diffs)
    print("mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
