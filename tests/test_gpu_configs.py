"""GPU: BASELINE configs 2 and 5 at their scaled bounds, and the exhaustible
rungs below them.

* Config 2 (standard-raft, Value = {v1, v2}, MaxElections = 3:
  configs/Raft_n3v2e3.cfg; Raft.tla:243 gates RequestVote on electionCtr) and
  config 5 scaled (RaftFsync, Value = {v1, v2}, MaxElections = 3,
  MaxRestarts = 1: configs/RaftFsync_n3v2e3r1.cfg; Restart truncates to
  fsyncIndex, RaftFsync.tla:203-218) are beyond one GPU's capacity, so they
  are pinned level by level (tests/golden/ladders.json): the C oracle to the
  first level boundary past 2*10^7 distinct states, its first 12 levels also
  reproduced by the literal Python oracle.  The GPU runs exactly that many
  levels (max_depth) and must match every (generated, new) pair and the
  hidden-variable collisions, single-shard, with 2 logical shards, and with 4
  logical shards each keeping its levels in host pages.  Config 3
  (FlexibleRaft.cfg verbatim, N = 5) likewise, to the first level boundary
  past 10^7 distinct states.
* The exhaustible rungs -- the bench workload Raft_n3v2e2 (1.885 * 10^9
  distinct), RaftFsync_n3v1e2r1 (6.3 * 10^8) and config 5's largest rung a
  node holds, RaftFsync_n3v1e2r2 (1.126 * 10^9) -- are checked in full:
  counts equal to the committed record (tests/golden/exhausted.json, made by
  tools/make_exhausted_record.py), its first levels equal to both oracles',
  64-bit == 128-bit fingerprints, 2 logical shards == 1, host frontier ==
  device frontier, and the first 25 levels equal to the CPU engine's.
"""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LAD = json.load(open(os.path.join(HERE, "golden", "ladders.json")))
EXH = json.load(open(os.path.join(HERE, "golden", "exhausted.json")))
BEYOND = ["raft_n3v2e3_cfg2", "fsync_n3v2e3r1_cfg5", "flex_cfg3"]

pytestmark = pytest.mark.gpu


def model(g):
    return raftmc.Model(module=g["module"], cfg_path=os.path.join(ROOT, g["cfg_path"]))


def prefix_match(r, g):
    assert r["levels"] == g["levels"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["status"] == "stopped"
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(LAD))
def test_ladder_prefix_matches_oracle(name):
    g = LAD[name]
    prefix_match(model(g).check(max_depth=g["depth"]), g)


@pytest.mark.parametrize("name", BEYOND)
def test_ladder_prefix_logical_shards(name):
    g = LAD[name]
    prefix_match(model(g).check_logical(2, max_depth=g["depth"]), g)


@pytest.mark.parametrize("name", BEYOND)
def test_ladder_prefix_host_frontier(name):
    g = LAD[name]
    prefix_match(model(g).check(max_depth=g["depth"], host_frontier=1), g)


@pytest.mark.parametrize("name", BEYOND)
def test_ladder_prefix_sharded_host_frontiers(name):
    """The configs beyond one GPU the way they are run at scale: fingerprint-
    sharded (4 logical shards), every shard's levels in host pages."""
    g = LAD[name]
    prefix_match(model(g).check_logical(4, max_depth=g["depth"], host_frontier=1), g)


_full = {}


def full(name):
    if name not in _full:
        _full[name] = model(EXH[name]).check()
    return _full[name]


def same(r, e):
    for k in ("generated", "distinct", "depth", "status", "levels", "hidden_var_collisions"):
        assert r[k] == e[k], (k, r["status"], r.get("message"))


@pytest.mark.parametrize("name", sorted(EXH))
def test_rung_exhaustive_record(name):
    e = EXH[name]
    r = full(name)
    same(r, e)
    k = e["oracle_levels"]
    # the C oracle's run over the rung (tools/fold_oracle_rungs.py), else the ladder prefix of both oracles
    pinned = e["oracle"]["levels"] if "oracle" in e else LAD.get(name, {}).get("levels", [])
    assert r["levels"][:k] == pinned[:k]


@pytest.mark.parametrize("name", sorted(EXH))
def test_rung_fp128_equals_fp64(name):
    want = full(name)
    raftmc.release_device_memory()  # the 128-bit set (32 B entries) needs the HBM the 64-bit one cached
    same(model(EXH[name]).check(fp_bits=128), want)


@pytest.mark.parametrize("name", sorted(EXH))
def test_rung_two_logical_shards(name):
    same(model(EXH[name]).check_logical(2), full(name))


@pytest.mark.parametrize("name", sorted(EXH))
def test_rung_host_frontier(name):
    want = full(name)
    raftmc.release_device_memory()
    same(model(EXH[name]).check(host_frontier=1), want)


@pytest.mark.parametrize("name", sorted(EXH))
def test_rung_cpu_engine_prefix(name):
    r = model(EXH[name]).check_cpu(max_depth=25)
    assert r["levels"] == full(name)["levels"][:25]


def test_per_shard_device_memory_scales_with_shards():
    """The sharded search partitions the state-proportional memory: on the
    bench rung (1.885e9 states) the HBM each logical shard holds at the end of
    the check (rmc_result.device_bytes: fingerprint set, frontiers, trace
    records, candidate scratch) is <= 0.6 of the single-GPU search's at W = 2
    and <= 0.35 at W = 4, with every count equal."""
    g = EXH["raft_n3v2e2_bench"]
    cfg = os.path.join(ROOT, g["cfg_path"])
    m = raftmc.Model(module=g["module"], cfg_path=cfg)
    single = m.check()
    assert (single["distinct"], single["generated"], single["depth"]) == (g["distinct"], g["generated"], g["depth"])
    for W, bound in ((2, 0.6), (4, 0.35)):
        # the same model: both searches pack rows to the message count the first
        # check measured (a fresh single-GPU check widens its rows to it in place;
        # the sharded search starts a fresh model at the constants-based default)
        r = m.check_logical(W)
        assert (r["distinct"], r["generated"], r["depth"]) == (g["distinct"], g["generated"], g["depth"])
        assert r["device_bytes"] <= bound * single["device_bytes"], (W, r["device_bytes"], single["device_bytes"])


# ---- r06: config 5's R-ladder at V = 1, E = 2 (tests/golden/fsync_rladder.json)
RL = json.load(open(os.path.join(HERE, "golden", "fsync_rladder.json")))


def _rmodel(R):
    return raftmc.Model(module="RaftFsync", cfg_path=os.path.join(ROOT, "configs", "RaftFsync_n3v1e2r%d.cfg" % R))


def test_fsync_r3_exhausts_and_its_prefix_equals_the_c_oracle():
    """RaftFsync_n3v1e2r3 in full on one GPU: the recorded totals, and every
    one of its first 38 levels equal to the C oracle's own run of them."""
    r = _rmodel(3).check()
    g = RL["gpu"]["r3"]
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    ol = RL["oracle_r3_levels"]
    assert r["levels"][:len(ol)] == ol


@pytest.mark.parametrize("R", [4, 7])
def test_fsync_r_ladder_saturates(R):
    """Every R >= 3 gives R = 3's 1,179,899,717 distinct states (restartCtr is
    outside VIEW): the R-ladder cannot be sized to a node."""
    r = _rmodel(R).check()
    g = RL["gpu"]["r%d" % R]
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (g["generated"], g["distinct"], g["depth"], "ok")
    assert r["distinct"] == RL["gpu"]["r3"]["distinct"]
