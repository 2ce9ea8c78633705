"""The CPU engine (rmc_check_cpu: TLC -workers N on host threads, BASELINE.md's
CPU baseline) against the oracle fixtures.  CPU only: it runs the same packed
layout, lowered actions, fingerprint and first-in-TLC-order rule as the GPU
path, so it must reproduce every count, the hidden-variable collision counts
and the counts at a violation, for any number of workers and chunk size."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))
UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))
N5 = json.load(open(os.path.join(HERE, "golden", "n5.json")))


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(SMALL))
@pytest.mark.parametrize("workers,chunk", [(1, 0), (4, 0), (3, 17)])
def test_cpu_engine_small(name, workers, chunk):
    g = SMALL[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_cpu(workers=workers, chunk_parents=chunk), g)


@pytest.mark.parametrize("name", ["fsync_n2v1e3_order", "fsync_n2v2e1r1_hidden"])
@pytest.mark.parametrize("workers,chunk", [(1, 0), (8, 0), (5, 999)])
def test_cpu_engine_first_wins(name, workers, chunk):
    """TLC-order-sensitive fixtures: counts and hidden-variable collisions."""
    g = ORDER[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_cpu(workers=workers, chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(UNSAFE))
@pytest.mark.parametrize("workers,chunk", [(1, 0), (6, 7)])
def test_cpu_engine_violation_counts(name, workers, chunk):
    g = UNSAFE[name]
    r = raftmc.Model(module=g["module"], cfg_text=g["cfg"]).check_cpu(workers=workers, chunk_parents=chunk)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert len(r["trace"]) == g["trace_len"] and r["trace"][0][0] == "Initial predicate"


@pytest.mark.parametrize("name", ["flex_n5v1e1_eq3rq4", "pull_n5v1e1"])
def test_cpu_engine_n5_levels(name):
    g = N5[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    depth = 0 if g["status"] == "ok" else min(g["depth"], 16)
    r = m.check_cpu(workers=8, max_depth=depth)
    assert r["levels"] == g["levels"][:len(r["levels"])] and len(r["levels"]) == (depth or g["depth"])


def test_cpu_engine_medium_violation():
    """RaftFsync with FollowerFsyncBeforeReply=FALSE (RaftFsync.tla:14-24): the
    counts at the first violating state in TLC order, per level."""
    g = MEDIUM["fsync_n3v1e2_unsafe"]
    r = raftmc.Model(module=g["module"], cfg_text=g["cfg"]).check_cpu(workers=8)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert len(r["trace"]) == g["trace_len"]


def test_cpu_engine_refuses_checkpoint(tmp_path):
    """Snapshots are the GPU search's (rmc_check); the CPU engine says so instead of ignoring them."""
    g = SMALL["raft_n3v1e1"]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    with pytest.raises(raftmc.RaftmcError, match="checkpoint"):
        m.check_cpu(checkpoint_dir=tmp_path)


EXTRAS = json.load(open(os.path.join(HERE, "golden", "extras.json")))


@pytest.mark.parametrize("name", sorted(EXTRAS))
def test_cpu_engine_classic_invariants(name):
    """The opt-in classic Raft properties (ElectionSafety, LogMatching,
    LeaderCompleteness, StateMachineSafety): both oracles' outcome."""
    g = EXTRAS[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.check_cpu(workers=4)
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    if g["status"] == "violation":
        assert r["violated"] == g["violated"] and len(r["trace"]) == g["trace_len"]
    else:
        assert r["levels"] == g["levels"]
