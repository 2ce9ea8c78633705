"""GPU parity: the HIP path (librmc via its C ABI) against the oracle's fixtures.

Counts must match bit-exactly: states generated, distinct states, depth and
every per-level (generated, new) pair.  Fixtures: tests/golden/small.json
(Python oracle == C oracle) and tests/golden/shipped.json (C oracle on the
reference's shipped cfgs).
"""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
SHIPPED_PATH = os.path.join(HERE, "golden", "shipped.json")
SHIPPED = json.load(open(SHIPPED_PATH)) if os.path.exists(SHIPPED_PATH) else {}

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(SMALL))
def test_small_configs_match_oracle(name):
    g = SMALL[name]
    r = raftmc.check_text(g["module"], g["cfg"])
    assert r["status"] == g["status"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(SMALL)[:3])
def test_tiny_chunks_and_table_growth(name):
    """Many chunks per level and a table that must grow: same counts."""
    g = SMALL[name]
    r = raftmc.check_text(g["module"], g["cfg"], chunk_parents=7, frontier_cap=64)
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]


@pytest.mark.parametrize("name", sorted(SHIPPED))
def test_shipped_configs_match_oracle(name):
    g = SHIPPED[name]
    r = raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"])).check()
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]
    assert r["status"] == "ok"
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(SHIPPED))
def test_tight_rows_from_the_previous_check(name):
    """The largest |DOMAIN messages| the GPU materializes equals the oracle's;
    a second check of the same model packs rows to exactly that many message
    slots (smaller rows) and must reproduce every count."""
    g = SHIPPED[name]
    m = raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"]))
    r1 = m.check()
    assert r1["max_msgs"] == g["max_msgs"]
    r2 = m.check()
    assert r2["state_bytes"] <= r1["state_bytes"]
    words = (1 + 4 * N_SERVERS[g["module"]] + g["max_msgs"] + 3) // 4 * 4  # rows are 16 B multiples
    assert r2["state_bytes"] == 4 * words
    assert (r2["generated"], r2["distinct"], r2["depth"], r2["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert r2["max_msgs"] == g["max_msgs"]


N_SERVERS = {"Raft": 3, "PullRaft": 3, "RaftFsync": 3, "FlexibleRaft": 5, "PullRaftVariant2": 3}


def test_report_is_tlc_format():
    g = SMALL["raft_n3v1e1"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    m.check()
    rep = m.report()
    assert "Model checking completed. No error has been found." in rep
    assert "%d states generated, %d distinct states found, 0 states left on queue." % (
        g["generated"], g["distinct"]) in rep
    assert "The depth of the complete state graph search is %d." % g["depth"] in rep


MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))


@pytest.mark.parametrize("name", sorted(k for k in MEDIUM if MEDIUM[k]["status"] == "ok"))
def test_medium_configs_match_oracle(name):
    g = MEDIUM[name]
    r = raftmc.check_text(g["module"], g["cfg"])
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(k for k in MEDIUM if MEDIUM[k]["status"] == "violation"))
@pytest.mark.parametrize("chunk", [0, 1000])
def test_violation_found_with_trace(name, chunk):
    """An unsafe config (RaftFsync.tla:14-24 policy) must report the same
    invariant, at the same depth, with a behaviour that starts at Init, and
    TLC's counts at the first violating state in TLC order (Appendix A.7: the
    counts at a violation are comparable in TLC order)."""
    g = MEDIUM[name]
    r = raftmc.check_text(g["module"], g["cfg"], chunk_parents=chunk)
    assert r["status"] == "violation"
    assert r["violated"] == g["violated"]
    tr = r["trace"]
    assert tr[0][0] == "Initial predicate"
    assert len(tr) == g["trace_len"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]


UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))


@pytest.mark.parametrize("name", sorted(UNSAFE))
@pytest.mark.parametrize("chunk", [0, 9])
def test_unsafe_flexible_violation(name, chunk):
    """Non-intersecting Flexible quorums: same invariant, same depth, a trace of
    the oracle's length, and the oracle's counts at the first violating state
    in TLC order."""
    g = UNSAFE[name]
    r = raftmc.check_text(g["module"], g["cfg"], chunk_parents=chunk)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert r["depth"] == g["depth"] and len(r["trace"]) == g["trace_len"]
    assert r["trace"][0][0] == "Initial predicate"
    assert (r["generated"], r["distinct"]) == (g["generated"], g["distinct"])
