"""GPU: Next as the TLA+ front end lowers it --
reordered, reduced, or with DuplicateMessage / DropMessage re-enabled
(Raft.tla:540-541) -- run by the HIP kernels through the C ABI
(rmc_model_set_next is the front end's output form; the .tla texts
themselves need the reference, so tests/test_frontend.py checks text ->
table on the CPU).  Every count, level and hidden-variable collision equals
the Python oracle with the same Next (tests/golden/frontend.json), in one
chunk, in small chunks, with two logical shards and with 128-bit
fingerprints."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
FRONTEND = json.load(open(os.path.join(HERE, "golden", "frontend.json")))

pytestmark = pytest.mark.gpu


def model(g):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    m.set_next(g["next"])
    return m


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (
        g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(FRONTEND))
@pytest.mark.parametrize("chunk", [0, 37])
def test_lowered_next_matches_oracle(name, chunk):
    g = FRONTEND[name]
    same(model(g).check(max_depth=g["max_depth"], chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(FRONTEND))
def test_lowered_next_two_logical_shards(name):
    g = FRONTEND[name]
    same(model(g).check_logical(2, max_depth=g["max_depth"]), g)


@pytest.mark.parametrize("name", ["raft_dup_n3v1e2", "raft_reversed_n2v2e2r1", "pull2_drop_reversed_n3v1e1"])
def test_lowered_next_fp128(name):
    g = FRONTEND[name]
    same(model(g).check(max_depth=g["max_depth"], fp_bits=128), g)
