"""Capacity model: does BASELINE config 2 (Raft, N=3, V=2, MaxElections=3) fit
one GPU, or 8?  Validated extrapolation of a BFS's level sizes.

Method.  Past the first ~15 levels the level-to-level growth ratio
r_k = n_{k+1} / n_k of these Raft state spaces falls almost linearly with the
depth k until the levels shrink to nothing.  Fit r_k = a + b k
by least squares on a window of known levels, extend the levels with the
fitted ratios while r > 0 (and n >= 1), and sum.  The fit is VALIDATED on the
two BASELINE rungs that do exhaust (their full level lists are in
tests/golden/exhausted.json): cut each at the same depth as config 2's known
prefix, predict, and compare the prediction with the true total, peak level
and depth.  The validation errors give the band applied to config 2.

    python tools/capacity_model.py > profiles/r05/capacity_model.txt
"""
import json
import math
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fit_line(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    sxy = sum((x - mx) * (y - my) for x, y in zip(xs, ys))
    b = sxy / sxx
    return my - b * mx, b


def fit_quad(xs, ys):
    # least squares for y = a + b x + c x^2 (normal equations, 3x3)
    import numpy as np
    A = np.array([[1.0, x, x * x] for x in xs])
    coef, *_ = np.linalg.lstsq(A, np.array(ys, dtype=float), rcond=None)
    return coef


def extrapolate(levels, window, kind):
    """levels: new-state counts per depth (depth 1 = levels[0]).  Returns
    (total distinct, peak level size, peak depth, last depth)."""
    n = list(map(float, levels))
    K = len(n)
    ks = list(range(K - window, K))  # ratio r_k = n[k] / n[k-1] for depth k+1
    rs = [n[k] / n[k - 1] for k in ks]
    if kind == "linear":
        a, b = fit_line(ks, rs)
        r = lambda k: a + b * k  # noqa: E731
    else:
        c0, c1, c2 = fit_quad(ks, rs)
        r = lambda k: c0 + c1 * k + c2 * k * k  # noqa: E731
    k = K
    cur = n[-1]
    while k < 400:
        rk = r(k)
        if rk <= 0:
            break
        cur *= rk
        if cur < 1:
            break
        n.append(cur)
        k += 1
    peak = max(range(len(n)), key=lambda i: n[i])
    return sum(n), n[peak], peak + 1, len(n)


def ladder(path):
    """Per-level new states from a verbose ladder log ("[rmc] depth d: n new, ...")."""
    txt = open(os.path.join(ROOT, path)).read()
    lv = {1: 1}
    for d, new in re.findall(r"depth (\d+): (\d+) new", txt):
        lv[int(d)] = int(new)
    return [lv[d] for d in range(1, max(lv) + 1)]


# The BASELINE configs and rungs that do NOT exhaust on one GPU, with the
# deepest prefix measured (the ladder logs under profiles/).
TARGETS = [
    ("config 2: Raft N=3 V=2 E=3 R=0 (configs/Raft_n3v2e3.cfg)",
     "profiles/r04/ladder_Raft_n3v2e3_hf1_compact.txt", 112),
    ("config 3: FlexibleRaft.cfg verbatim, N=5 EQ=3 RQ=4 V=2 E=2 (configs/FlexibleRaft.cfg)",
     "profiles/r03/ladder_FlexibleRaft_hf1.txt", 160),
    ("config 5 rung: RaftFsync N=3 V=2 E=2 R=1 (configs/RaftFsync_n3v2e2r1.cfg)",
     "profiles/r03/ladder_RaftFsync_n3v2e2r1_hf1.txt", 112),
    ("config 5 scaled: RaftFsync N=3 V=2 E=3 R=1 (configs/RaftFsync_n3v2e3r1.cfg)",
     "profiles/r02/ladder_RaftFsync_n3v2e3r1.txt", 112),
    # r06: the R-ladder at V=1, E=2 saturates at R=3 (1,179,899,717 distinct for
    # every R >= 3, profiles/r06/ladder5/); the next RaftFsync rungs are R=0 on
    # the V and E axes
    ("config 5 rung: RaftFsync N=3 V=2 E=2 R=0 (configs/RaftFsync_n3v2e2.cfg)",
     "profiles/r06/ladder5/RaftFsync_n3v2e2.txt", 112),
    ("config 5 rung: RaftFsync N=3 V=1 E=3 R=0 (configs/RaftFsync_n3v1e3.cfg)",
     "profiles/r06/ladder5/RaftFsync_n3v1e3.txt", 112),
]
EXTRA = os.environ.get("CAPACITY_EXTRA", "")  # "label|path|row_bytes;..." rungs measured later


def main():
    ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exhausted.json")))
    cuts = (25, 27, 29, 31, 33)
    windows = (4, 6, 8, 10, 14)
    print("Capacity model (tools/capacity_model.py): linear fit of the level growth ratio r_k = n_{k+1}/n_k")
    print("on the last W known levels, extended until r <= 0 or a level falls below one state.")
    print("(A quadratic fit of r_k was tried too: on these prefixes it curves back up and diverges -- unusable.)")
    print()
    print("Validation on the two rungs that exhaust (tests/golden/exhausted.json), cut at depths %s:" % (cuts,))
    errs = {}
    for name, g in sorted(ex.items()):
        full = [x[1] for x in g["levels"]]
        true_total, true_peak = sum(full), max(full)
        true_pd = full.index(true_peak) + 1
        print("  %s: actual %d distinct, peak level %d states at depth %d, depth %d" %
              (name, true_total, true_peak, true_pd, len(full)))
        for cut in cuts:
            row = []
            for W in windows:
                tot, pk, pd, last = extrapolate(full[:cut], W, "linear")
                errs.setdefault(W, []).append(tot / true_total)
                row.append("W=%-2d x%.2f" % (W, tot / true_total))
            print("    cut at depth %d: predicted total / actual:  %s" % (cut, "  ".join(row)))
    print()
    best = min(errs, key=lambda W: max(abs(math.log(e)) for e in errs[W]))
    lo, hi = min(errs[best]), max(errs[best])
    print("Best window on the validation rungs: W=%d, predicted/actual total within x%.2f .. x%.2f over %d cuts." %
          (best, lo, hi, len(errs[best])))
    hbm = 288e9
    cap = {e: hbm / e * 0.75 for e in (16, 8)}
    print("One MI355X's fingerprint set (288 GB at 0.75 load): %.2e states at 16 B per entry, %.2e at 8 B; "
          "an 8-GPU node: %.2e / %.2e." % (cap[16], cap[8], 8 * cap[16], 8 * cap[8]))
    targets = list(TARGETS)
    for item in filter(None, EXTRA.split(";")):
        label, path, rb = item.split("|")
        targets.append((label, path, int(rb)))
    for label, path, row_bytes in targets:
        lv = ladder(path)
        print()
        print("%s, known to depth %d (%s: %d distinct states):" % (label, len(lv), path, sum(lv)))
        for W in windows:
            tot, pk, pd, last = extrapolate(lv, W, "linear")
            print("  W=%-2d: %.3e distinct, peak level %.3e at depth %d, depth %d%s" %
                  (W, tot, pk, pd, last, "  <- validated best" if W == best else ""))
        tot, pk, pd, last = extrapolate(lv, best, "linear")
        band = (tot / hi, tot / lo)  # truth = prediction / (predicted/actual)
        mid = math.sqrt(band[0] * band[1])
        peak = pk / math.sqrt(lo * hi)
        print("  Estimate: ~%.1e distinct states (band %.1e .. %.1e), a peak level of ~%.1e states near depth %d, "
              "depth ~%d." % (mid, band[0], band[1], peak, pd, last))
        for e in (16, 8):
            print("    fingerprint set at %2d B per entry: needs %.1f..%.1f GPUs' HBM (an 8-GPU node holds %.2e)"
                  % (e, band[0] / cap[e], band[1] / cap[e], 8 * cap[e]))
        print("    the peak level at %d B per compact row: %.2f TB (8 x 288 GB of HBM = 2.3 TB; host pages 8 x 270 GiB = "
              "2.3 TB)" % (row_bytes, peak * row_bytes / 1e12))
        fits = band[1] <= 8 * cap[8]
        print("    -> %s" % ("fits an 8-GPU node's fingerprint sets (8 B entries) even at the band's top" if fits else
                            "fits an 8-GPU node only if the truth is near the band's bottom" if band[0] <= 8 * cap[8]
                            else "out of reach of an 8-GPU node by a factor of %.0f at the band's bottom (8 B entries)"
                            % (band[0] / (8 * cap[8]))))


if __name__ == "__main__":
    main()
