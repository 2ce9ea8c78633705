"""GPU: random simulation (TLC -simulate) through the C ABI.

Simulation is random, so there are no oracle counts to match; what is pinned:
known-unsafe configs yield the oracle's violated invariant with a behaviour
that the independent Python oracle replays from its own Init through its own
Next (every step must be one of the oracle's successors, as TLC would check a
-dumpTrace module) and whose last state violates the invariant under the
oracle, a safe config yields none, a seed reproduces its run exactly, and
the counters are consistent (every behaviour contributes 1..depth+1 states).
"""
import json
import os

import pytest

import raftmc
from oracle.pyoracle import make_spec, parse_cfg
from test_gpu_trace import _final_oracle_state
from test_trace_module import parse_trace_states

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))
N5 = json.load(open(os.path.join(HERE, "golden", "n5.json")))

pytestmark = pytest.mark.gpu


UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))


@pytest.mark.parametrize("name", sorted(UNSAFE))
def test_simulation_finds_unsafe_flexible_violation(name):
    """Non-intersecting Flexible quorums: random behaviours find the oracle's
    violated invariant; the behaviour replays from Init (at least as long as
    the BFS-shortest counterexample)."""
    g = UNSAFE[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.simulate(walkers=1 << 14, depth=60, seed=7, behaviors=1 << 22, seconds=60)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    tr = r["trace"]
    assert tr[0][0] == "Initial predicate" and len(tr) >= g["trace_len"]
    # the behaviour, as the -dumpTrace module holds it, replayed by the oracle
    tla, _ = m.trace_module(g["module"] + "_STrace")
    states = parse_trace_states(tla)
    assert len(states) == len(tr)
    spec = make_spec(g["module"], parse_cfg(g["cfg"]))
    last = _final_oracle_state(spec, states)
    assert not dict(spec.invariants)[g["violated"]](last)


def test_simulation_violation_replays_in_oracle_n5():
    """Five servers with election quorums of 2 (n5.json): a simulated violation
    of the 120-permutation model, replayed step by step by the oracle."""
    g = N5["flex_n5v1e2_eq2rq2_unsafe"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.simulate(walkers=1 << 14, depth=60, seed=9, behaviors=1 << 22, seconds=60)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    tla, _ = m.trace_module(g["module"] + "_STrace")
    states = parse_trace_states(tla)
    spec = make_spec(g["module"], parse_cfg(g["cfg"]))
    last = _final_oracle_state(spec, states)
    assert not dict(spec.invariants)[g["violated"]](last)


@pytest.mark.parametrize("name", ["raft_n3v1e1", "pull_n3v2e1", "flex_n3v1e1", "fsync_n3v1e1"])
def test_simulation_safe_configs(name):
    g = SMALL[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    depth, behaviors = 50, 1 << 16
    r = m.simulate(walkers=1 << 14, depth=depth, seed=3, behaviors=behaviors)
    assert r["status"] == "ok"
    assert r["behaviors"] == behaviors
    assert behaviors < r["generated"] <= behaviors * (depth + 1)
    assert 2 <= r["depth"] <= depth + 1


def test_simulation_is_reproducible_per_seed():
    g = SMALL["raft_n3v1e1r1"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    a = m.simulate(walkers=4096, depth=40, seed=11, behaviors=20000)
    b = m.simulate(walkers=4096, depth=40, seed=11, behaviors=20000)
    c = m.simulate(walkers=4096, depth=40, seed=12, behaviors=20000)
    assert (a["generated"], a["depth"]) == (b["generated"], b["depth"])
    assert a["generated"] != c["generated"]


@pytest.mark.parametrize("name", sorted(UNSAFE))
def test_simulation_violation_is_reproducible(name):
    """The reported failure is the lowest-index failing behaviour of the round
    and every behaviour runs to its end, so the counts and the trace at a
    violation are a function of the seed (not of wave scheduling)."""
    g = UNSAFE[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    runs = [m.simulate(walkers=1 << 14, depth=60, seed=5, behaviors=1 << 20) for _ in range(3)]
    assert runs[0]["status"] == "violation"
    for r in runs[1:]:
        assert (r["generated"], r["behaviors"], r["depth"], r["violated"]) == \
            (runs[0]["generated"], runs[0]["behaviors"], runs[0]["depth"], runs[0]["violated"])
        assert r["trace"] == runs[0]["trace"]
