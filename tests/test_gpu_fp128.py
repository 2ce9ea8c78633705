"""GPU: 128-bit fingerprints (fp_bits=128; SURVEY.md §7 hard part 2 asks for a
wider mode because min-over-permutations raises the collision rate).  The
first 64 bits are the 64-bit fingerprint, the second word an independent hash
of the same canonical view (tests/test_lowering.py pins incremental == full
for both words on every successor of the small configs).  Every count must
equal the oracles' -- far below 2^32 states a 64-bit collision is negligible,
so both widths must agree exactly -- including TLC-order-sensitive fixtures,
hidden-variable collisions, violation counts and the grow / redo paths."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))
N5 = json.load(open(os.path.join(HERE, "golden", "n5.json")))

pytestmark = pytest.mark.gpu


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(SMALL))
def test_fp128_small(name):
    g = SMALL[name]
    same(raftmc.check_text(g["module"], g["cfg"], fp_bits=128), g)


@pytest.mark.parametrize("name", sorted(ORDER))
@pytest.mark.parametrize("chunk", [0, 500])
def test_fp128_first_wins(name, chunk):
    g = ORDER[name]
    same(raftmc.check_text(g["module"], g["cfg"], fp_bits=128, chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(k for k in MEDIUM))
def test_fp128_medium(name):
    g = MEDIUM[name]
    r = raftmc.check_text(g["module"], g["cfg"], fp_bits=128)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    if g["status"] == "violation":
        assert r["violated"] == g["violated"] and len(r["trace"]) == g["trace_len"]


@pytest.mark.parametrize("name", ["flex_n5v1e1_eq3rq4", "raft_n5v1e1"])
def test_fp128_n5(name):
    g = N5[name]
    r = raftmc.check_text(g["module"], g["cfg"], fp_bits=128, max_depth=g["depth"])
    assert r["levels"] == g["levels"]


@pytest.mark.parametrize("name", ["pull_n3v1e2r1", "raft_n4v1e1"])
def test_fp128_overflow_redo(name):
    g = MEDIUM[name]
    r = raftmc.check_text(g["module"], g["cfg"], fp_bits=128, hash_slots=64, grow_on_overflow=True, chunk_parents=777)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])


def test_fp128_rejected_where_not_offered():
    g = SMALL["raft_n3v1e1"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    with pytest.raises(raftmc.RaftmcError, match="128"):
        m.check_logical(2, fp_bits=128)
