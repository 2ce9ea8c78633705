"""GPU parity at N=5 (the k_expand<*,5> / k_materialize<*,5> instantiations and
the 120-permutation canonical fingerprint, FlexibleRaft.cfg's server count).

Fixtures (tests/golden/n5.json, tests/cfgs.py N5): level-truncated runs of the C
oracle (exhaustive N=5 runs take it hours), the first 12-22 levels also
reproduced by the literal Python oracle.  The GPU runs exactly the fixture's
number of levels (max_depth) and must match every per-level (generated, new)
pair bit for bit, single-shard and through the sharded protocol.
"""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
N5 = json.load(open(os.path.join(HERE, "golden", "n5.json")))
CASES = sorted(k for k in N5 if N5[k]["status"] in ("ok", "truncated"))
UNSAFE = sorted(k for k in N5 if N5[k]["status"] == "violation")

pytestmark = pytest.mark.gpu


def levels_match(r, g):
    assert r["levels"] == g["levels"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["status"] == ("ok" if g["status"] == "ok" else "stopped")


@pytest.mark.parametrize("name", CASES)
def test_n5_levels_match_oracle(name):
    g = N5[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.check(max_depth=0 if g["status"] == "ok" else g["depth"])
    levels_match(r, g)
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", CASES[:3])
def test_n5_small_chunks(name):
    """Many k_expand launches per level (chunk boundaries inside 5-server levels)."""
    g = N5[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    levels_match(m.check(max_depth=0 if g["status"] == "ok" else g["depth"], chunk_parents=3000), g)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("shards", [3])
def test_n5_logical_shards(name, shards):
    g = N5[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    levels_match(m.check_logical(shards, max_depth=0 if g["status"] == "ok" else g["depth"]), g)


@pytest.mark.parametrize("name", UNSAFE)
def test_n5_unsafe_violation(name):
    """5 servers with election quorums of 2 (not intersecting; FlexibleRaft.tla:16-24
    lists the valid pairs): the oracle's invariant, depth and trace length."""
    g = N5[name]
    r = raftmc.check_text(g["module"], g["cfg"])
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert r["depth"] == g["depth"] and len(r["trace"]) == g["trace_len"]
    assert r["trace"][0][0] == "Initial predicate"
    assert (r["generated"], r["distinct"]) == (g["generated"], g["distinct"])
    assert r["levels"] == g["levels"]
