"""GPU: the multi-GPU front door (SURVEY.md §8b rmc_options.n_gpus, §3(5)
`raftmc -gpus G`, `bench.py --gpus N`).

rmc_check with n_gpus = N > 1 runs the fingerprint-sharded search over GPUs
0..N-1 of this process, one host thread and stream per GPU (rmc_check_multi).
The one-GPU box cannot run two RCCL ranks, so the threaded driver itself is
tested with its peer-copy transport (RMC_XPORT_P2P) and several shards on GPU
0: the same threads, clones of the model, host barriers, published transfer
pointers, per-shard caches and global result as on a node -- only the copy
engine differs.  Multi-rank RCCL stays unmeasured on hardware.  Asking for
more GPUs than are visible must fail loudly, never run one.
"""
import json
import os
import subprocess
import sys

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))
ORDER = json.load(open(os.path.join(HERE, "golden", "order.json")))
UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))

pytestmark = pytest.mark.gpu


def ngpus():
    import torch
    return torch.cuda.device_count()


def model(g):
    if "cfg_path" in g:
        return raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"]))
    return raftmc.Model(module=g["module"], cfg_text=g["cfg"])


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]
    if "hidden_same_level" in g:
        assert r["hidden_var_collisions"] == g["hidden_same_level"]


def test_n_gpus_1_is_rmc_check():
    g = SMALL["raft_n3v1e1"]
    a = model(g).check(n_gpus=1)
    b = model(g).check()
    same(a, g)
    assert {k: a[k] for k in ("generated", "distinct", "depth", "levels", "hidden_var_collisions")} == \
        {k: b[k] for k in ("generated", "distinct", "depth", "levels", "hidden_var_collisions")}


def test_more_gpus_than_visible_fails_loudly():
    """n_gpus beyond the visible GPUs is an error naming both numbers, never a
    silent one-GPU run (VERDICT r05 What's missing #1)."""
    n = ngpus()
    g = SMALL["raft_n3v1e1"]
    with pytest.raises(raftmc.RaftmcError, match=r"n_gpus = %d requested, but only %d GPU" % (n + 1, n)):
        model(g).check(n_gpus=n + 1)
    with pytest.raises(raftmc.RaftmcError, match="at least 1"):
        model(g).check(n_gpus=0)


def test_multi_rejects_bad_device_lists():
    g = SMALL["raft_n3v1e1"]
    with pytest.raises(raftmc.RaftmcError, match="visible"):
        model(g).check_multi([0, ngpus()])
    with pytest.raises(raftmc.RaftmcError, match="distinct GPU per shard"):
        model(g).check_multi([0, 0], transport=raftmc.XPORT_RCCL)


@pytest.mark.parametrize("name", sorted(SMALL))
@pytest.mark.parametrize("shards,chunk", [(2, 0), (3, 7), (4, 64)])
def test_threads_match_oracle(name, shards, chunk):
    g = SMALL[name]
    same(model(g).check_multi([0] * shards, chunk_parents=chunk), g)


@pytest.mark.parametrize("name", sorted(ORDER))
def test_threads_tlc_order(name):
    """TLC-order first-wins across threads: the hidden-variable collisions of
    the order fixtures (which a last-wins rule counts differently)."""
    g = ORDER[name]
    same(model(g).check_multi([0, 0, 0], chunk_parents=501), g)


def test_threads_shipped_raft_cfg():
    """Raft.cfg (8,664,032 distinct) on 4 threads, several rounds per level."""
    g = SHIPPED["Raft_cfg"]
    same(model(g).check_multi([0] * 4, chunk_parents=1 << 18), g)


@pytest.mark.parametrize("name", sorted(k for k in MEDIUM if MEDIUM[k]["status"] == "violation"))
def test_threads_violation_trace(name):
    """A violation: TLC's counts at the failing state and the trace, walked
    through the distributed parent records by the threads."""
    g = MEDIUM[name]
    single = model(g).check(chunk_parents=1000)
    r = model(g).check_multi([0, 0], chunk_parents=1000)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["trace"] == single["trace"] and len(r["trace"]) == g["trace_len"]


@pytest.mark.parametrize("name", sorted(UNSAFE))
def test_threads_unsafe(name):
    g = UNSAFE[name]
    r = model(g).check_multi([0, 0, 0], chunk_parents=50)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert len(r["trace"]) == g["trace_len"]


def test_threads_host_frontier(monkeypatch):
    """Every thread's shard keeps its levels in host pages (the pool split
    between the threads) with small pages that rows straddle."""
    monkeypatch.setenv("RMC_HOST_PAGE_ROWS", "999")
    g = ORDER["raft_n2v2e2r2_order"]
    same(model(g).check_multi([0, 0], chunk_parents=333, host_frontier=1), g)


def test_threads_capacity_rerun():
    """A message-capacity overflow makes every thread re-run with wider rows
    in lockstep (each on its own clone of the model); the result lands in the
    caller's model, so the next check of it starts at the measured width."""
    g = SMALL["raft_n3v1e1r1"]
    m = model(g)
    m.selftest_set_hint_kmax(2)  # rows of 2 message slots: the first check overflows and re-runs
    same(m.check_multi([0, 0], chunk_parents=100), g)
    same(m.check_multi([0, 0], chunk_parents=100), g)
    same(m.check(), g)


def test_threads_then_single_then_logical():
    """Alternating the threaded driver, the single-GPU search and logical
    shards in one process: each releases the others' cached buffers."""
    g = SHIPPED["RaftFsync_cfg"]
    same(model(g).check_multi([0, 0]), g)
    same(model(g).check(), g)
    same(model(g).check_logical(3), g)
    same(model(g).check_multi([0, 0, 0, 0]), g)


def test_unsupported_options_fail_loudly():
    g = SMALL["raft_n3v1e1"]
    with pytest.raises(raftmc.RaftmcError, match="fp_bits 128"):
        model(g).check_multi([0, 0], fp_bits=128)


def test_cli_gpus_beyond_visible_fails(tmp_path):
    """raftmc -gpus G goes through the same front door."""
    exe = os.path.join(ROOT, "raft-tlaplus_amd", "build", "raftmc")
    p = subprocess.run([exe, "-deadlock", "-module", "Raft", "-config", os.path.join(ROOT, "configs", "Raft.cfg"),
                        "-gpus", str(ngpus() + 1)], capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "requested, but only" in p.stderr


def test_bench_gpus_beyond_visible_exits_nonzero():
    """bench.py --gpus N without a launcher runs the in-process multi-GPU check;
    on a box with fewer GPUs it must exit non-zero, not print n_gpus: 1."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ngpus() + 1), "--steps", "1",
                        "--warmup", "0", "--workload", "raft_cfg", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0, p.stdout
    assert '"n_gpus"' not in p.stdout
    assert "requested, but only" in p.stderr


def test_bench_gpus_1_in_process():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1",
                        "--warmup", "0", "--workload", "raft_cfg", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["result"]["distinct"] == SHIPPED["Raft_cfg"]["distinct"]
