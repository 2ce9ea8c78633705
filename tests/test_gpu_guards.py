"""GPU: Next with actions behind compiled guards (SURVEY.md §8f rank 4;
rmc_guard.cpp -> rmc_spec.h guard_vm run inside k_expand), through the C ABI
(rmc_model_set_guard is the table a module with an edited guard lowers to;
the .tla texts need the reference, so tests/test_guards.py checks text ->
guard on the CPU).  Every count, level and hidden-variable collision equals
the Python oracle with the same guard (tests/golden/guards.json), in one
chunk, in small chunks, with two logical shards and with the host frontier."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
GUARDS = json.load(open(os.path.join(HERE, "golden", "guards.json")))

pytestmark = pytest.mark.gpu


def model(g):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    for action, params, expr in g["guards"]:
        m.set_guard(action, params, expr)
    return m


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (
        g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(GUARDS))
@pytest.mark.parametrize("chunk", [0, 37])
def test_compiled_guards_match_oracle(name, chunk):
    g = GUARDS[name]
    same(model(g).check(max_depth=g["max_depth"], chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(GUARDS))
def test_compiled_guards_two_logical_shards(name):
    g = GUARDS[name]
    same(model(g).check_logical(2, max_depth=g["max_depth"]), g)


@pytest.mark.parametrize("name", ["raft_quant_n2v1e2", "fsync_timeout_rvij_n2v1e2r1"])
def test_compiled_guards_host_frontier(name):
    g = GUARDS[name]
    same(model(g).check(max_depth=g["max_depth"], host_frontier=1), g)


def test_compiled_guards_refuse_fp128():
    g = GUARDS["raft_rv_le_n2v1e1"]
    with pytest.raises(raftmc.RaftmcError, match="64-bit"):
        model(g).check(fp_bits=128)
