"""GPU: BFS levels in pinned host memory (rmc_options.host_frontier, raftmc
-hostfrontier; SURVEY.md §7 hard part 5 and step 8).  The current and next
level live in host pages and stream through double-buffered HBM windows, so
the fingerprint set can take the whole device.  Whatever the mode -- always
on the host, switched to the host in the middle of a level (the auto mode's
reaction to HBM running out: before a chunk, or when the next level's buffer
cannot grow), tiny pages that rows straddle -- every count, per-level pair,
hidden-variable collision count, violation and trace must equal the oracle
fixtures and the device-frontier search."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))
UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))

pytestmark = pytest.mark.gpu


def model(g):
    if "cfg_path" in g:
        return raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"]))
    return raftmc.Model(module=g["module"], cfg_text=g["cfg"])


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(SMALL))
def test_always_host_small(name):
    g = SMALL[name]
    same(model(g).check(host_frontier=1, chunk_parents=500), g)


@pytest.mark.parametrize("name", sorted(ORDER))
def test_always_host_tlc_order(name):
    """TLC-order first-wins fixtures: chunks stream through alternating windows."""
    g = ORDER[name]
    same(model(g).check(host_frontier=1, chunk_parents=777), g)


def test_always_host_small_pages(monkeypatch):
    """Pages of 1,000 rows: chunks and output batches straddle many pages, and
    consumed pages are recycled while the level is read."""
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "1000")
    g = SHIPPED["Raft_cfg"]
    same(model(g).check(host_frontier=1, chunk_parents=30000), g)


@pytest.mark.parametrize("how", ["", ":grow"])
@pytest.mark.parametrize("level", [12, 30])
def test_auto_switch_mid_level(monkeypatch, how, level):
    """Auto mode moving the frontiers to the host in the middle of a level:
    before a chunk (as when the set cannot grow), or with a chunk expanded
    and marked but not yet materialized (the next level's buffer cannot grow)."""
    monkeypatch.setenv("RMC_HOST_FRONTIER_AT", "%d%s" % (level, how))
    g = SHIPPED["Raft_cfg"]
    same(model(g).check(host_frontier=0, chunk_parents=20000), g)


def test_never_host_is_unchanged(monkeypatch):
    monkeypatch.setenv("RMC_HOST_FRONTIER_AT", "12")
    g = SHIPPED["Raft_cfg"]
    same(model(g).check(host_frontier=-1, chunk_parents=20000), g)


@pytest.mark.parametrize("fp_bits", [64, 128])
def test_always_host_shipped(fp_bits):
    g = SHIPPED["RaftFsync_cfg"]
    same(model(g).check(host_frontier=1, fp_bits=fp_bits), g)


VIOL = dict(UNSAFE)
VIOL.update({k: v for k, v in MEDIUM.items() if v["status"] == "violation"})


@pytest.mark.parametrize("name", sorted(VIOL))
@pytest.mark.parametrize("chunk", [9, 1000, 0])
def test_always_host_violation(name, chunk):
    """A violation found with the host frontier: TLC's counts at the failing
    state (its chunk re-expanded from the host pages) and the same trace."""
    g = VIOL[name]
    dev = model(g).check(chunk_parents=chunk)
    r = model(g).check(host_frontier=1, chunk_parents=chunk)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["trace"] == dev["trace"] and len(r["trace"]) == g["trace_len"]


def test_host_checkpoint_and_recover(tmp_path):
    """Snapshots written from host pages; a resumed check on the host frontier."""
    g = SHIPPED["Raft_cfg"]
    a = model(g).check(host_frontier=1, max_depth=20, checkpoint_dir=tmp_path, checkpoint_minutes=0)
    assert a["status"] == "stopped"
    same(model(g).check(host_frontier=1, recover_dir=tmp_path), g)
    same(model(g).check(recover_dir=tmp_path), g)


def test_host_frontier_in_the_sharded_search_too():
    """r04: the sharded search takes the option per shard (tests/test_gpu_sharded.py has its cases)."""
    g = SMALL["raft_n3v1e1"]
    same(model(g).check_logical(2, host_frontier=1), g)


@pytest.mark.parametrize("frac", ["0.0000001", "0.00002"])
def test_auto_switch_at_a_level_boundary(monkeypatch, frac):
    """The auto mode's level-boundary switch (a next level projected past a
    fraction of HBM moves both levels to the host before the level starts):
    RMC_HF_HBM_FRACTION lowers the quarter-of-HBM threshold so it fires on
    Raft.cfg -- at the first levels, or deeper -- and the counts equal the
    device-frontier search's and the oracle's."""
    monkeypatch.setenv("RMC_HF_HBM_FRACTION", frac)
    g = SHIPPED["Raft_cfg"]
    same(model(g).check(host_frontier=0, chunk_parents=50000), g)


@pytest.mark.parametrize("name", ["fsync_n2v2e2r1_hidden", "raft_n2v2e2r2_order"])
def test_auto_switch_tlc_order(monkeypatch, name):
    monkeypatch.setenv("RMC_HF_HBM_FRACTION", "0.000001")
    g = ORDER[name]
    same(model(g).check(host_frontier=0, chunk_parents=333), g)


@pytest.mark.parametrize("shards", [0, 2])
def test_row_length_bound_reports_capacity(monkeypatch, shards):
    """r05 regression for the r04 driver fault: a compact row's length comes
    from its header, and k_row_words bounds it by the row width instead of
    letting k_pack_rows and the copy-out run past their buffers.
    RMC_HF_ROW_MAX_WORDS lowers the bound below real rows (header + 1
    message), so the bound fires on the first level with two messages: the
    check ends with status "capacity" and the completed levels, a prefix of
    the fixture's, instead of faulting."""
    g = SMALL["raft_n3v1e1"]
    monkeypatch.setenv("RMC_HF_ROW_MAX_WORDS", str(1 + 4 * 3 + 1))
    m = model(g)
    r = m.check_logical(shards, host_frontier=1) if shards else m.check(host_frontier=1)
    assert r["status"] == "capacity", (r["status"], r.get("message"))
    assert "exceeds the row width" in r["message"]
    k = len(r["levels"])
    assert 1 <= k < len(g["levels"])
    assert r["levels"] == g["levels"][:k]  # the level that met the bound is not counted
    assert r["distinct"] == sum(n for _, n in g["levels"][:k])


def test_back_to_back_host_checks_reuse_pinned_pages(monkeypatch):
    """r05: pinned pages outlive a check (a process-wide cache) and a page given
    up is never unmapped, so back-to-back host-frontier checks in one process
    -- the GPU suite's pattern, ~30 of them, when the r04 driver run faulted in
    a copy-out -- register no address twice."""
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "2000")
    for name in ("fsync_n3v1e2_unsafe", "flex_n3v2e2_eq1"):
        g = VIOL[name]
        for chunk in (0, 1000, 0):
            r = model(g).check(host_frontier=1, chunk_parents=chunk)
            assert r["status"] == "violation" and (r["generated"], r["distinct"]) == (g["generated"], g["distinct"])


def test_pack_buffer_regrows_while_copy_outs_run(monkeypatch):
    """r06, the r05 fault's named path driven on purpose (VERDICT r05 What's
    weak #3): with 7-parent chunks a chunk's new rows outgrow the compact-row
    pack buffer of its output window (sized for 3 rows per parent) while the
    previous same-parity chunk's copy-out may still read it.  The regrowth
    waits for that copy-out's event and then checks (hipEventQuery) that no
    copy stream still uses the buffer -- a missing wait is an error naming the
    buffer, not a GPU fault.  Small pages make the rows straddle pages."""
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "64")
    regrows = 0
    for name in ("raft_n2v2e2r2_order", "fsync_n2v2e2r1_hidden"):
        g = ORDER[name]
        m = model(g)
        same(m.check(host_frontier=1, chunk_parents=7), g)
        regrows += m.selftest_hf_stats()[0]
    g = SMALL["raft_n3v1e1r1"]
    m = model(g)
    same(m.check(host_frontier=1, chunk_parents=7), g)
    regrows += m.selftest_hf_stats()[0]
    assert regrows >= 1


def test_first_check_phases_add_up():
    """rmc_check_phases: the named phases of a check are non-negative and
    their sum stays within the total."""
    g = SHIPPED["Raft_cfg"]
    m = model(g)
    m.check(chunk_parents=20000)
    p = m.phases()
    assert set(p) >= {"hip_init", "buffers", "launch_enqueue", "table_growth", "kernels", "total"}
    assert all(v >= 0 for v in p.values())
    # (hip_init precedes the check's own clock; launch enqueue overlaps kernels)
    # (sub-phases "a.b" are parts of phase a)
    assert sum(v for k, v in p.items() if k not in ("total", "hip_init") and "." not in k) <= p["total"] * 1.2 + 0.05
    parts = [v for k, v in p.items() if k.startswith("table_growth.")]
    assert len(parts) == 3 and sum(parts) <= p["table_growth"] + 1e-6
