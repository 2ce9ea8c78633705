"""GPU: rows widened in place mid-check (r05, VERDICT r04 "tight rows from the
first check").  A model checked for the first time starts with rows for N
message slots; a chunk whose successors need more widens the current level's
rows and the next level's rows so far, resets the ranks its first attempt
claimed (the message bindings' TLC ordinals depend on the slot count) and is
redone.  Whatever the chunk size -- widenings at the first chunk of a level or
in the middle of one -- every count, per-level pair, hidden-variable
collision count, violation and trace must equal the oracle fixtures and the
check at a fixed capacity."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))
UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))
EXHAUSTED = json.load(open(os.path.join(HERE, "golden", "exhausted.json")))

pytestmark = pytest.mark.gpu


def model(g):
    if "cfg_path" in g:
        return raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"]))
    return raftmc.Model(module=g["module"], cfg_text=g["cfg"])


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("chunk", [0, 20000, 777])
def test_fresh_model_widens_mid_level(chunk):
    """Raft.cfg (8.6M states, up to ~30 messages per state): a fresh model
    widens several times, some of them in the middle of a multi-chunk level;
    the counts equal the fixture, and the next check of the same model starts
    at the measured width (no widening)."""
    g = SHIPPED["Raft_cfg"]
    m = model(g)
    r = m.check(chunk_parents=chunk)
    same(r, g)
    w = m.selftest_widenings()
    assert len(w) >= 3, w
    if chunk == 777:
        assert any(c0 > 0 for _, c0, _ in w), w  # at least one chunk redone mid-level
    assert r["max_msgs"] <= w[-1][2]
    r2 = m.check(chunk_parents=chunk)
    same(r2, g)
    assert m.selftest_widenings() == []
    assert r2["state_bytes"] == r["state_bytes"]


@pytest.mark.parametrize("name", sorted(ORDER))
def test_widening_keeps_tlc_order_first_wins(name):
    """The TLC-order fixtures (hidden-variable collisions decided by the
    ordinals) with widenings in the middle of levels."""
    g = ORDER[name]
    m = model(g)
    same(m.check(chunk_parents=97), g)


@pytest.mark.parametrize("name", sorted(SMALL))
def test_widening_small_fixtures_fp128(name):
    g = SMALL[name]
    same(model(g).check(chunk_parents=300, fp_bits=128), g)


@pytest.mark.parametrize("name", sorted(UNSAFE))
def test_widening_violation_counts_and_trace(name):
    g = UNSAFE[name]
    m = model(g)
    r = m.check(chunk_parents=50)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert len(r["trace"]) == g["trace_len"]
    # the whole behaviour -- action labels and states -- equals a
    # check at a fixed capacity (no widening), so trace records written before
    # a widening (old binding numbering) are replayed correctly
    w = m.selftest_widenings()
    fixed = model(g).check(chunk_parents=50, msg_cap_K=40)
    assert fixed["trace"] == r["trace"], w


def test_bench_rung_fresh_model_equals_exhausted():
    """The bench workload checked by a fresh model: widened from 7 message
    slots to its maximum, all 69 levels equal the committed full record
    (pinned by the C oracle's full run)."""
    e = EXHAUSTED["raft_n3v2e2_bench"]
    m = model(e)
    r = m.check()
    for k in ("generated", "distinct", "depth", "status", "levels", "hidden_var_collisions"):
        assert r[k] == e[k], (k, r["status"], r.get("message"))
    assert r["state_bytes"] == 192  # 13 header words + 35 message slots: the tight row
    assert len(m.selftest_widenings()) >= 3


def test_widening_mid_level_then_violation_trace():
    """At least one UNSAFE case widens in the middle of a level (c0 > 0) before
    the violating level; its trace equals the fixed-capacity check's."""
    hits = 0
    for name in sorted(UNSAFE):
        g = UNSAFE[name]
        m = model(g)
        r = m.check(chunk_parents=7)
        w = m.selftest_widenings()
        assert r["status"] == "violation"
        if any(c0 > 0 and d < r["depth"] for d, c0, _ in w):
            hits += 1
            assert model(g).check(chunk_parents=7, msg_cap_K=40)["trace"] == r["trace"]
    assert hits >= 1
