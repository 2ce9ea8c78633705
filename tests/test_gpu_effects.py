"""GPU: Next with actions the TLA+ front end compiles whole -- guard and
effect (rmc_guard.cpp compile_effect -> rmc_spec.h
effect_vm run inside k_expand and k_materialize) -- through the C ABI
(rmc_model_define_action + rmc_model_set_next is the table a module with such
a Next disjunct lowers to; the .tla texts need the reference, so
tests/test_effects.py checks module text -> compiled action on the CPU).
Every count, level, hidden-variable collision and violated invariant equals
the Python oracle with the same actions (tests/golden/effects.json), in one
chunk, in small chunks, with two logical shards and with the host frontier;
a violation's trace ends in a state the compiled action produced."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
EFFECTS = json.load(open(os.path.join(HERE, "golden", "effects.json")))

pytestmark = pytest.mark.gpu


def model(g):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    for name, form, params, body in g["actions"]:
        m.define_action(name, form, params, body)
    m.set_next(g["next"])
    return m


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (
        g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]
    if g["status"] == "violation":
        assert r["violated"] == g["violated"]


@pytest.mark.parametrize("name", sorted(EFFECTS))
@pytest.mark.parametrize("chunk", [0, 37])
def test_compiled_actions_match_oracle(name, chunk):
    g = EFFECTS[name]
    same(model(g).check(max_depth=g["max_depth"], chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(EFFECTS))
def test_compiled_actions_two_logical_shards(name):
    g = EFFECTS[name]
    same(model(g).check_logical(2, max_depth=g["max_depth"]), g)


@pytest.mark.parametrize("name", ["raft_rv_noself_n3v1e2", "fsync_rvij_empty_n2v1e2r1"])
def test_compiled_actions_host_frontier(name):
    g = EFFECTS[name]
    same(model(g).check(max_depth=g["max_depth"], host_frontier=1), g)


def test_compiled_action_violation_trace():
    """ClientRequestEager acks at once: LeaderHasAllAckedValues breaks, and
    the trace names the compiled action on the way there."""
    g = EFFECTS["raft_client_eager_n3v1e2"]
    m = model(g)
    r = m.check()
    assert r["status"] == "violation" and r["violated"] == "LeaderHasAllAckedValues"
    tr = m.trace()
    assert len(tr) == g["depth"]
    assert any("ClientRequestEager" in step[0] for step in tr)
