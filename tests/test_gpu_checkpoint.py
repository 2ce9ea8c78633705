"""GPU: TLC's -checkpoint / -recover (the reference's
states/ directory, .gitignore:1).  A check stopped after some levels with a
snapshot at every level boundary, then resumed from the snapshot, must give
exactly the counts, per-level pairs, hidden-variable collisions and (at a
violation) the counts and trace of an uninterrupted check."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
V2 = json.load(open(os.path.join(HERE, "golden", "variant2.json")))
UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))

pytestmark = pytest.mark.gpu


def model(g):
    if "cfg_path" in g:
        return raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"]))
    return raftmc.Model(module=g["module"], cfg_text=g["cfg"])


CASES = [("shipped", "Raft_cfg"), ("order", "fsync_n2v2e2r1_hidden"), ("v2", "pull2_n3v1e2r1")]
TABLES = {"shipped": SHIPPED, "order": ORDER, "v2": V2}


@pytest.mark.parametrize("table,name", CASES)
@pytest.mark.parametrize("fp_bits", [64, 128])
def test_stop_snapshot_resume(tmp_path, table, name, fp_bits):
    g = TABLES[table][name]
    stop_at = max(2, g["depth"] // 2)
    a = model(g).check(max_depth=stop_at, checkpoint_dir=tmp_path, checkpoint_minutes=0, fp_bits=fp_bits)
    assert a["status"] == "stopped" and a["depth"] == stop_at
    assert (tmp_path / "checkpoint.meta").exists()
    r = model(g).check(recover_dir=tmp_path, fp_bits=fp_bits)
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


def test_resume_then_snapshot_again(tmp_path):
    """A resumed check takes snapshots too: three legs reach the uninterrupted result."""
    g = SHIPPED["Raft_cfg"]
    d1, d2 = tmp_path / "a", tmp_path / "b"
    model(g).check(max_depth=10, checkpoint_dir=d1, checkpoint_minutes=0)
    model(g).check(max_depth=20, recover_dir=d1, checkpoint_dir=d2, checkpoint_minutes=0)
    r = model(g).check(recover_dir=d2)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])


@pytest.mark.parametrize("name", sorted(UNSAFE))
def test_resume_finds_the_violation(tmp_path, name):
    """Resumed before the violating level: the same violation, counts at it and trace."""
    g = UNSAFE[name]
    full = model(g).check()
    model(g).check(max_depth=max(2, g["depth"] - 3), checkpoint_dir=tmp_path, checkpoint_minutes=0)
    r = model(g).check(recover_dir=tmp_path)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["trace"] == full["trace"]


def test_recover_refuses_another_model(tmp_path):
    g = SHIPPED["Raft_cfg"]
    model(g).check(max_depth=5, checkpoint_dir=tmp_path, checkpoint_minutes=0)
    other = ORDER["raft_n2v2e2r2_order"]
    with pytest.raises(raftmc.RaftmcError, match="different model"):
        model(other).check(recover_dir=tmp_path)
    with pytest.raises(raftmc.RaftmcError, match="no checkpoint"):
        model(g).check(recover_dir=tmp_path / "missing")


def test_resume_overflows_message_capacity(tmp_path):
    """A snapshot packed with fewer message slots than later levels need: the
    resumed check overflows the capacity after the resume level, re-runs from
    the same snapshot with more slots (its rows widened on load) and reaches the
    uninterrupted result -- it neither loops on the snapshot nor fails."""
    g = SHIPPED["Raft_cfg"]
    m = model(g)
    m.selftest_set_hint_kmax(8)
    a = m.check(max_depth=12, checkpoint_dir=tmp_path, checkpoint_minutes=0)
    assert a["status"] == "stopped" and a["depth"] == 12
    snap_slots = a["state_bytes"] // 4 - 1 - 4 * 3
    assert snap_slots < g["max_msgs"]  # the resumed levels cannot fit the snapshot's rows
    r = model(g).check(recover_dir=tmp_path)
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["levels"] == g["levels"]
    assert r["state_bytes"] // 4 - 1 - 4 * 3 >= g["max_msgs"]


def test_snapshot_replaces_the_previous_one(tmp_path):
    """Each snapshot goes to a fresh subdirectory named by checkpoint.meta; the
    previous one is removed only after the new one is complete."""
    g = SHIPPED["Raft_cfg"]
    model(g).check(max_depth=8, checkpoint_dir=tmp_path, checkpoint_minutes=0)
    subs = sorted(p.name for p in tmp_path.iterdir() if p.is_dir())
    assert len(subs) == 1 and subs[0].startswith("snap-")
    assert sorted(p.name for p in (tmp_path / subs[0]).iterdir()) == \
        ["fpset.bin", "frontier.bin", "trace_bind.bin", "trace_parent.bin"]
    assert "snapshot %s" % subs[0][len("snap-"):] in (tmp_path / "checkpoint.meta").read_text()
    r = model(g).check(recover_dir=tmp_path)
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])


@pytest.mark.parametrize("width_change", [False, True])
def test_recover_into_host_pages(tmp_path, monkeypatch, width_change):
    """A snapshot taken with the levels on the host (RMC_HOST_FRONTIER_AT moves
    them there mid-level) and resumed with a small frontier_cap: the saved level
    streams from the file straight into pinned host pages (RMC_RECOVER_TO_HOST
    stands for "past the auto switch's threshold"), the device frontiers are
    never sized for it, and the result equals the uninterrupted check -- also
    when the resumed level overflows the snapshot's message capacity (rows
    widened on the way into the pages)."""
    g = SHIPPED["Raft_cfg"]
    m = model(g)
    if width_change:
        m.selftest_set_hint_kmax(8)
    monkeypatch.setenv("RMC_HOST_FRONTIER_AT", "12")
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "4099")
    a = m.check(max_depth=16, checkpoint_dir=tmp_path, checkpoint_minutes=0, chunk_parents=20000)
    assert a["status"] == "stopped" and a["depth"] == 16
    monkeypatch.delenv("RMC_HOST_FRONTIER_AT")
    monkeypatch.setenv("RMC_RECOVER_TO_HOST", "1")
    r = model(g).check(recover_dir=tmp_path, frontier_cap=1 << 10, chunk_parents=30000)
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


def test_stale_snapshots_are_removed(tmp_path):
    """Snapshot directories the meta does not name (an interrupted rotation, an
    earlier model's snapshot) are removed at the next snapshot."""
    g = SHIPPED["Raft_cfg"]
    (tmp_path / "snap-77").mkdir()
    (tmp_path / "snap-77" / "fpset.bin").write_bytes(b"x" * 100)
    model(g).check(max_depth=6, checkpoint_dir=tmp_path, checkpoint_minutes=0)
    subs = sorted(p.name for p in tmp_path.iterdir() if p.is_dir())
    assert len(subs) == 1 and subs[0] != "snap-77"
