"""GPU: TLC-order first-wins under VIEW, hidden-variable collision counts, and
the fingerprint set's growth / redo / message-capacity safety nets.

VIEW view drops acked, electionCtr and restartCtr (Raft.tla:115), which gate
ClientRequest (:306) and RequestVote (:243): two successors with one view but
different hidden values can have different futures, and TLC keeps the one it
generated first (SURVEY.md §7 hard part 1).  tests/golden/order.json holds
configs where this happens; for three of them the C oracle's --reverse-order
probe (the LAST successor in TLC order wins) gives different counts, so only
the exact first-in-TLC-order winner reproduces them.  The GPU must also count
the same-level collisions exactly as the oracles do (hidden_same_level).
"""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))

pytestmark = pytest.mark.gpu


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(ORDER))
def test_first_in_tlc_order_wins(name):
    g = ORDER[name]
    r = raftmc.check_text(g["module"], g["cfg"])
    same(r, g)
    rv = g["reverse_order"]
    if (rv["generated"], rv["distinct"]) != (g["generated"], g["distinct"]):
        # the fixture discriminates: a wrong winner would have produced these
        assert (r["generated"], r["distinct"]) != (rv["generated"], rv["distinct"])


@pytest.mark.parametrize("name", sorted(ORDER))
@pytest.mark.parametrize("chunk", [7, 1000])
def test_first_wins_across_chunks(name, chunk):
    """Same-level duplicates split over many k_expand launches."""
    g = ORDER[name]
    same(raftmc.check_text(g["module"], g["cfg"], chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(ORDER))
@pytest.mark.parametrize("shards,chunk", [(2, 0), (3, 13)])
def test_first_wins_across_shards(name, shards, chunk):
    g = ORDER[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_logical(shards, chunk_parents=chunk), g)


@pytest.mark.parametrize("name", ["pull_n3v1e2r1", "raft_n4v1e1"])
def test_fpset_grows_from_tiny(name):
    """The fingerprint set starts at 2^10 slots and must double many times ahead of chunks."""
    g = MEDIUM[name]
    r = raftmc.check_text(g["module"], g["cfg"], hash_slots=1 << 10)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert r["hash_capacity"] > 1 << 10


@pytest.mark.parametrize("name", ["pull_n3v1e2r1", "raft_n4v1e1"])
@pytest.mark.parametrize("chunk", [0, 333])
def test_fpset_overflow_redo(name, chunk):
    """A 64-slot set and no growth ahead of chunks: chunks overflow it, the
    driver grows it and redoes the chunk (inserts are idempotent); counts unchanged."""
    g = MEDIUM[name]
    r = raftmc.check_text(g["module"], g["cfg"], hash_slots=64, grow_on_overflow=True, chunk_parents=chunk)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", ["raft_n3v1e1", "pull_n3v2e1", "fsync_n3v1e1"])
def test_message_capacity_rerun(name):
    """Rows packed to fewer message slots than the model needs (as if the last
    check had seen fewer): the overflow takes the re-run path with a larger
    capacity and reproduces every count."""
    g = SMALL[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    m.selftest_set_hint_kmax(max(1, g["max_msgs"] - 6))
    r = m.check()
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert r["max_msgs"] == g["max_msgs"]


@pytest.mark.parametrize("name", ["fsync_n2v2e2r1_hidden", "raft_n2v2e2r2_order"])
@pytest.mark.parametrize("fp_bits", [64, 128])
def test_first_wins_through_redos(name, fp_bits):
    """Chunks redone after the fingerprint set overflows: the TLC-order winners
    and the hidden-variable collision count (a redone chunk's collisions
    counted once) are unchanged."""
    g = ORDER[name]
    same(raftmc.check_text(g["module"], g["cfg"], hash_slots=256, grow_on_overflow=True, chunk_parents=300,
                           fp_bits=fp_bits), g)
