"""Run the C oracle over a whole (or a deep prefix of a) BASELINE rung and record
its per-level counts.  TEST INFRASTRUCTURE ONLY (container CPU, hours).

    python tools/oracle_exhaust.py configs/RaftFsync_n3v1e2r1.cfg --fp-slots 800000000 \
        --out profiles/r04/oracle_RaftFsync_n3v1e2r1.json [--max-distinct N] [--threads 8]

The oracle streams its levels through files under oracle/_runs/ (--spill-dir)
and keeps a 16 B-per-slot fingerprint set; per-level progress goes to
<out>.log.  The JSON written at the end carries every level's (generated, new)
pair, the totals, the hidden-variable collisions and the wall time; a fixture
writer (tools/make_exhausted_record.py) folds it into tests/golden/exhausted.json.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import run_c  # noqa: E402
from oracle.pyoracle.cfg import parse_cfg  # noqa: E402

MODULE_OF = {"Raft": "Raft", "RaftFsync": "RaftFsync", "FlexibleRaft": "FlexibleRaft", "PullRaft": "PullRaft",
             "PullRaftVariant2": "PullRaftVariant2"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("--out", required=True)
    ap.add_argument("--fp-slots", type=int, default=0)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--max-distinct", type=int, default=0)
    a = ap.parse_args()
    base = os.path.basename(a.cfg)[:-4]
    module = MODULE_OF[base.split("_")[0]]
    cfg = parse_cfg(open(os.path.join(ROOT, a.cfg)).read())
    spill = os.path.join(ROOT, "oracle", "_runs", base)
    os.makedirs(spill, exist_ok=True)
    cmd = [run_c.BIN] + run_c.cfg_args(module, cfg["constants"], cfg["invariants"]) + \
        ["--threads", str(a.threads), "--no-trace", "--progress", "--spill-dir", spill]
    if a.fp_slots:
        cmd += ["--fp-slots", str(a.fp_slots)]
    if a.max_distinct:
        cmd += ["--max-distinct", str(a.max_distinct)]
    t0 = time.time()
    with open(a.out + ".log", "w") as log:
        log.write(" ".join(cmd) + "\n")
        log.flush()
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=log, text=True, check=True)
    r = json.loads(p.stdout)
    r.update(module=module, cfg_path=a.cfg, command=" ".join(os.path.relpath(c, ROOT) if c.startswith(ROOT) else c
                                                                 for c in cmd), wall_s=time.time() - t0)
    with open(a.out, "w") as f:
        json.dump(r, f, indent=1, sort_keys=True)
    print(r["status"], r["generated"], r["distinct"], r["depth"], "%.0f s" % r["wall_s"])


if __name__ == "__main__":
    main()
