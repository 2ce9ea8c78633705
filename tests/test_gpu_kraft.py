"""GPU: KRaft (pull-raft/KRaft.tla) through the C ABI
against the oracle fixtures (tests/golden/kraft.json): every per-level count,
the counts and invariant at a violation (IllegalState with restarts), over
chunk sizes, 128-bit fingerprints and the fingerprint-sharded protocol; the
shipped cfg's constants against the oracle's first levels and the CPU engine."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
KR = json.load(open(os.path.join(HERE, "golden", "kraft.json")))
FULL = sorted(k for k in KR if KR[k]["status"] != "truncated" and not KR[k].get("slow"))

pytestmark = pytest.mark.gpu


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    if g["status"] == "ok":
        assert r["levels"] == g["levels"]
        assert r["hidden_var_collisions"] == g["hidden_same_level"]
    else:
        assert r["violated"] == g["violated"]


@pytest.mark.parametrize("name", FULL)
@pytest.mark.parametrize("chunk", [0, 7, 1000])
def test_kraft_matches_oracle(name, chunk):
    g = KR[name]
    same(raftmc.check_text("KRaft", g["cfg"], chunk_parents=chunk), g)


@pytest.mark.parametrize("name", ["kraft_n3v2e1", "kraft_n2v2e2"])
def test_kraft_fp128(name):
    g = KR[name]
    same(raftmc.check_text("KRaft", g["cfg"], fp_bits=128), g)


@pytest.mark.parametrize("name", ["kraft_n3v2e1", "kraft_n3v1e1r1"])
@pytest.mark.parametrize("shards,chunk", [(2, 0), (3, 55)])
def test_kraft_logical_shards(name, shards, chunk):
    g = KR[name]
    r = raftmc.Model(module="KRaft", cfg_text=g["cfg"]).check_logical(shards, chunk_parents=chunk)
    if g["status"] == "ok":
        same(r, g)
    else:  # the sharded protocol stops at the violating round: TLC's trace, not its counts at the stop
        assert r["status"] == "violation" and r["violated"] == g["violated"]
        assert r["depth"] == g["depth"] and len(r["trace"]) == g["trace_len"]


def test_kraft_violation_trace():
    """The IllegalState behaviour is rebuilt and ends in the violating state."""
    g = KR["kraft_n2v1e2r1"]
    m = raftmc.Model(module="KRaft", cfg_text=g["cfg"])
    r = m.check()
    assert r["status"] == "violation" and r["violated"] == "NoIllegalState"
    tr = m.trace()
    assert len(tr) == g["trace_len"]
    assert "IllegalState" in tr[-1][1]


def test_kraft_shipped_cfg():
    """KRaft.cfg's constants (19,841,847 distinct, 57,806,118 generated, depth
    52): every level equal to the C++ oracle's, and GPU == CPU engine."""
    g = KR["KRaft_cfg"]  # C++ oracle, exhaustive (its first 16 levels also the Python oracle's)
    m = raftmc.Model(module="KRaft", cfg_path=os.path.join(ROOT, "configs", "KRaft.cfg"))
    r = m.check()
    assert (r["generated"], r["distinct"], r["depth"], r["status"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"], g["levels"])
    assert r["hidden_var_collisions"] == g["hidden_same_level"]
    c = m.check_cpu(workers=16)
    assert (r["generated"], r["distinct"], r["depth"], r["status"], r["levels"]) == \
        (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"])


def test_kraft_simulation():
    """TLC -simulate on KRaft: restarts reach IllegalState (the replayed behaviour
    ends there); KRaft.cfg's constants (safe: exhausted above) find nothing."""
    g = KR["kraft_n3v1e1r1"]
    r = raftmc.Model(module="KRaft", cfg_text=g["cfg"]).simulate(walkers=1 << 14, depth=60, seed=3,
                                                                behaviors=1 << 20, seconds=60)
    assert r["status"] == "violation" and r["violated"] == "NoIllegalState"
    assert r["trace"][0][0] == "Initial predicate" and len(r["trace"]) >= g["trace_len"]
    assert "IllegalState" in r["trace"][-1][1]
    s = raftmc.Model(module="KRaft", cfg_path=os.path.join(ROOT, "configs", "KRaft.cfg")).simulate(
        walkers=1 << 14, depth=80, seed=5, behaviors=1 << 18)
    assert s["status"] == "ok" and s["behaviors"] == 1 << 18


def test_kraft_dump_trace_module():
    """TLC -dumpTrace tla: the IllegalState behaviour as a module over KRaft's variables."""
    g = KR["kraft_n2v1e2r1"]
    m = raftmc.Model(module="KRaft", cfg_text=g["cfg"])
    m.check()
    tla, cfg = m.trace_module("KRaftTrace")
    assert "EXTENDS KRaft" in tla and "pendingFetch |->" in tla and "IllegalState" in tla
