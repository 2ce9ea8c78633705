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

    python tools/capacity_model.py > profiles/r04/capacity_model.txt
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


def known_config2():
    """Config 2 per-level new states from the compact host-frontier ladder (depth 31 reached)."""
    txt = open(os.path.join(ROOT, "profiles", "r04", "ladder_Raft_n3v2e3_hf1_compact.txt")).read()
    lv = {1: 1}
    for d, new in re.findall(r"depth (\d+): (\d+) new", txt):
        lv[int(d)] = int(new)
    return [lv[d] for d in range(1, max(lv) + 1)]


def main():
    ex = json.load(open(os.path.join(ROOT, "tests", "golden", "exhausted.json")))
    c2 = known_config2()
    cut0 = len(c2)
    cuts = (25, 27, 29, 31, 33)
    windows = (4, 6, 8, 10, 14)
    print("Capacity model (tools/capacity_model.py): linear fit of the level growth ratio r_k = n_{k+1}/n_k")
    print("on the last W known levels, extended until r <= 0 or a level falls below one state.  Config 2 is known")
    print("to depth %d (profiles/r04/ladder_Raft_n3v2e3_hf1_compact.txt: %d distinct states)." % (cut0, sum(c2)))
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
    print()
    print("Config 2 (Raft_n3v2e3), known to depth %d:" % cut0)
    for W in windows:
        tot, pk, pd, last = extrapolate(c2, W, "linear")
        print("  W=%-2d: %.3e distinct, peak level %.3e at depth %d, depth %d%s" %
              (W, tot, pk, pd, last, "  <- validated best" if W == best else ""))
    tot, pk, pd, last = extrapolate(c2, best, "linear")
    band = (tot / hi, tot / lo)  # truth = prediction / (predicted/actual)
    mid = math.sqrt(band[0] * band[1])
    print()
    print("Estimate: config 2 has ~%.1e distinct states (band %.1e .. %.1e: the W=%d prediction %.2e divided by the "
          "validation's predicted/actual range), a peak level of ~%.1e states near depth %d, depth ~%d." %
          (mid, band[0], band[1], best, tot, pk / math.sqrt(lo * hi), pd, last))
    hbm = 288e9
    for entry in (16, 8):
        cap1 = hbm / entry * 0.75
        print("  fingerprint set, %2d B per entry at 0.75 load: 1 GPU holds %.2e states, 8 GPUs %.2e -> config 2 "
              "needs %.0f..%.0f GPUs' HBM for the set alone" % (entry, cap1, 8 * cap1, band[0] / cap1, band[1] / cap1))
    for S in (192.0, 112.0):
        print("  the peak level alone at %3.0f B per row: %.1f TB (8 x 288 GB of HBM = 2.3 TB; host pages: 8 x 270 GiB)"
              % (S, pk / math.sqrt(lo * hi) * S / 1e12))
    print("Conclusion: config 2 (MaxElections=3) is out of reach of one MI355X and of an 8-GPU node, by a factor of "
          "%.0f or more in fingerprint-set capacity alone at 8 B per entry." % (band[0] / (8 * hbm / 8 * 0.75)))


if __name__ == "__main__":
    main()
