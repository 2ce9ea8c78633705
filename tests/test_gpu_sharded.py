"""GPU: the fingerprint-sharded search (rmc_sharded.cpp) through the C ABI.

rmc_check_logical runs W shards of the multi-GPU protocol on this GPU (device
copies as the transport), so the exchange, owner dedupe, TLC-order first-wins
across shards and the block-cyclic redistribution are checked without a
cluster.  Counts must equal the oracle fixtures bit for
bit for every W and chunk size; a single-rank RCCL communicator exercises the
RCCL transport itself.
"""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))

pytestmark = pytest.mark.gpu


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]


@pytest.mark.parametrize("name", sorted(SMALL))
@pytest.mark.parametrize("shards,chunk", [(1, 0), (2, 0), (3, 7), (4, 64), (8, 5)])
def test_logical_shards_match_oracle(name, shards, chunk):
    g = SMALL[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_logical(shards, chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(k for k in MEDIUM if MEDIUM[k]["status"] == "ok"))
def test_logical_shards_medium(name):
    g = MEDIUM[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_logical(4, chunk_parents=4096), g)


def test_logical_shards_shipped_raft_cfg():
    g = SHIPPED["Raft_cfg"]
    m = raftmc.Model(module="Raft", cfg_path=os.path.join(ROOT, g["cfg_path"]))
    same(m.check_logical(8), dict(g, status="ok"))


@pytest.mark.parametrize("name", sorted(k for k in MEDIUM if MEDIUM[k]["status"] == "violation"))
@pytest.mark.parametrize("shards", [2, 5])
def test_logical_shards_violation_trace(name, shards):
    g = MEDIUM[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.check_logical(shards, chunk_parents=1000)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert r["trace"][0][0] == "Initial predicate"
    assert len(r["trace"]) == g["trace_len"]
    # TLC's counts at the failing state, as the single-shard search reports them
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]


def test_rccl_single_rank():
    g = SMALL["raft_n3v1e1"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_sharded(0, 1, 0, raftmc.comm_unique_id()), g)


def test_logical_growth_paths():
    """Tiny frontier capacity: the per-shard frontier and trace buffers grow mid-level."""
    g = SMALL["raft_n3v1e1r1"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_logical(3, chunk_parents=33, frontier_cap=16), g)


@pytest.mark.parametrize("name", ["pull_n3v1e2r1", "raft_n4v1e1"])
@pytest.mark.parametrize("shards,chunk", [(1, 0), (3, 333)])
def test_logical_table_overflow_redo(name, shards, chunk):
    """64-slot tables and no growth ahead of rounds: k_expand's local-owner
    inserts overflow a shard's table, every shard redoes the round after it
    grows; the owners' remote inserts grow the table mid-round (local-owner
    outcomes are then found by fingerprint).  Counts unchanged."""
    g = MEDIUM[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.check_logical(shards, chunk_parents=chunk, hash_slots=64, grow_on_overflow=True)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))


@pytest.mark.parametrize("name", sorted(UNSAFE))
@pytest.mark.parametrize("shards", [2, 3])
def test_logical_shards_unsafe(name, shards):
    g = UNSAFE[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.check_logical(shards, chunk_parents=50)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert r["depth"] == g["depth"] and len(r["trace"]) == g["trace_len"]
    assert (r["generated"], r["distinct"]) == (g["generated"], g["distinct"])


# ---- per-shard host frontier (rmc_options.host_frontier in the sharded search)
ORDER_HF = json.load(open(os.path.join(HERE, "golden", "order.json")))
SHIPPED_HF = json.load(open(os.path.join(HERE, "golden", "shipped.json")))


def _model(g):
    if "cfg_path" in g:
        return raftmc.Model(module=g["module"], cfg_path=os.path.join(os.path.dirname(HERE), g["cfg_path"]))
    return raftmc.Model(module=g["module"], cfg_text=g["cfg"])


def _same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(ORDER_HF))
@pytest.mark.parametrize("W", [2, 3])
def test_sharded_host_frontier_always(name, W, monkeypatch):
    """Every shard's levels in compact host pages (small pages, small rounds):
    the TLC-order fixtures' counts, levels and hidden-variable collisions."""
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "999")
    g = ORDER_HF[name]
    _same(_model(g).check_logical(W, host_frontier=1, chunk_parents=501), g)


def test_sharded_host_frontier_shipped_raft(monkeypatch):
    g = SHIPPED_HF["Raft_cfg"]
    _same(_model(g).check_logical(4, host_frontier=1, chunk_parents=100000), g)


def test_sharded_host_frontier_auto_switch(monkeypatch):
    """The auto mode's level-boundary switch, decided on the allgathered
    projections (RMC_HF_HBM_FRACTION lowers the threshold so it fires)."""
    monkeypatch.setenv("RMC_HF_HBM_FRACTION", "0.00002")
    g = SHIPPED_HF["Raft_cfg"]
    _same(_model(g).check_logical(2, host_frontier=0, chunk_parents=70000), g)


@pytest.mark.parametrize("shards", [0, 2])
def test_host_pages_exhausted_ends_with_the_completed_levels(monkeypatch, shards):
    """Host pages running out mid-level (RMC_HOST_FRONTIER_GIB far below the
    shipped Raft.cfg's levels, 1000-row pages) ends the check with status
    "capacity" and the counts of the levels completed before it, a prefix of
    the fixture's -- the single-GPU search and the sharded one alike."""
    monkeypatch.setenv("RMC_HOST_FRONTIER_GIB", "0.02")
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "1000")
    g = SHIPPED_HF["Raft_cfg"]
    m = _model(g)
    r = m.check_logical(shards, host_frontier=1) if shards else m.check(host_frontier=1)
    assert r["status"] == "capacity", (r["status"], r.get("message"))
    assert "host frontier pages exhausted" in r["message"]
    k = len(r["levels"])
    assert 3 < k < len(g["levels"])
    assert r["levels"] == g["levels"][:k]
    assert r["distinct"] == sum(n for _, n in g["levels"][:k])
    assert r["generated"] == sum(x for x, _ in g["levels"][:k])
