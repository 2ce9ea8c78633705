"""The oracle itself: pinned against SURVEY.md Appendix B (hand-derived first
BFS levels of each shipped cfg) and cross-checked between its two independent
restatements (literal Python, C).  CPU only."""
import json
import os

import pytest

from oracle import run_c
from oracle.pyoracle import make_spec
from oracle.pyoracle.cfg import ModelValue as MV, parse_cfg, load_cfg
from oracle.pyoracle.tlc import bfs, tlc_key, Rec
from cfgs import cfg_text

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="session", autouse=True)
def built_oracle():
    if not os.path.exists(run_c.BIN):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)


# (generated, new) for levels 1..3 of the shipped cfgs
APPENDIX_B = {
    "Raft": [(1, 1), (3, 1), (5, 3)],
    "PullRaft": [(1, 1), (3, 1), (5, 3)],
    "RaftFsync": [(1, 1), (3, 1), (5, 3)],
    "FlexibleRaft": [(1, 1), (5, 1), (9, 3)],
}


@pytest.mark.parametrize("module", sorted(APPENDIX_B))
def test_appendix_b_first_levels(module):
    cfg = load_cfg(os.path.join(ROOT, "configs", module + ".cfg"))
    r = bfs(make_spec(module, cfg), max_states=30)
    assert [tuple(x) for x in r.levels[:3]] == APPENDIX_B[module]


@pytest.mark.parametrize("module", sorted(APPENDIX_B))
def test_c_oracle_appendix_b(module):
    cfg = load_cfg(os.path.join(ROOT, "configs", module + ".cfg"))
    c = run_c.run(module, cfg["constants"], cfg["invariants"], extra=["--max-distinct", "20"])
    assert [tuple(x) for x in c["levels"][:3]] == APPENDIX_B[module]


@pytest.mark.parametrize("module,kw", [
    ("Raft", dict(n=2, v=1, E=2)), ("PullRaft", dict(n=3, v=1, E=1)),
    ("RaftFsync", dict(n=2, v=1, E=1, R=1)), ("FlexibleRaft", dict(n=2, v=1, E=2, ElectionQuorumSize=2,
                                                                  ReplicationQuorumSize=1)),
])
def test_python_and_c_oracles_agree(module, kw):
    txt = cfg_text(module, **kw)
    cfg = parse_cfg(txt)
    p = bfs(make_spec(module, cfg))
    c = run_c.run(module, cfg["constants"], cfg["invariants"])
    assert (p.generated, p.distinct, p.depth, p.status) == (c["generated"], c["distinct"], c["depth"], c["status"])
    assert [list(x) for x in p.levels] == c["levels"]


SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))


@pytest.mark.parametrize("name", sorted(SMALL))
def test_c_oracle_reproduces_fixture(name):
    g = SMALL[name]
    cfg = parse_cfg(g["cfg"])
    c = run_c.run(g["module"], cfg["constants"], cfg["invariants"], threads=2)
    assert (c["generated"], c["distinct"], c["depth"], c["levels"]) == (
        g["generated"], g["distinct"], g["depth"], g["levels"])


def test_c_oracle_threads_deterministic():
    g = SMALL["raft_n2v2e2"]
    cfg = parse_cfg(g["cfg"])
    a = run_c.run(g["module"], cfg["constants"], cfg["invariants"], threads=1)
    b = run_c.run(g["module"], cfg["constants"], cfg["invariants"], threads=8)
    assert a["levels"] == b["levels"] and a["distinct"] == b["distinct"]


def test_violation_trace_replays():
    """An unsafe RaftFsync config (FollowerFsyncBeforeReply=FALSE with restarts,
    RaftFsync.tla:14-24) violates LeaderHasAllAckedValues; the C oracle's trace
    must be a valid behaviour of the Python oracle's Next ending in the violation."""
    txt = cfg_text("RaftFsync", n=2, v=1, E=2, R=1, FollowerFsyncBeforeReply=False)
    cfg = parse_cfg(txt)
    c = run_c.run("RaftFsync", cfg["constants"], cfg["invariants"], extra=["--trace"])
    p = bfs(make_spec("RaftFsync", cfg))
    assert c["status"] == p.status
    if c["status"] == "violation":
        assert c["violated"] == p.violated
        assert len(c["trace"]) == len(p.trace)


def test_tlc_value_order():
    # records: field count first, then names/values interleaved (TLC RecordValue.compareTo)
    a = Rec(mtype="RequestVoteResponse", mterm=3, msource=1, mdest=0, mvoteGranted=True)
    b = Rec(mtype="RequestVoteRequest", mterm=1, mlastLogTerm=0, mlastLogIndex=0, msource=1, mdest=0)
    assert tlc_key(a) < tlc_key(b)  # 5 fields < 6 fields
    # same field count: "mlastLogIndex" < "mmatchIndex" decides after mdest
    c = Rec(mtype="AppendEntriesResponse", mterm=1, msuccess=False, mmatchIndex=0, msource=1, mdest=0)
    assert tlc_key(b) < tlc_key(c)
    assert tlc_key((1, 2)) > tlc_key((5,))  # sequences: length first


def test_cfg_quirks():
    txt = open(os.path.join(ROOT, "configs", "PullRaft.cfg")).read()
    cfg = parse_cfg(txt)
    assert cfg["constants"]["Value"] == frozenset([MV("v1"), MV("v2")])  # v2 never declared
    assert cfg["constants"]["n1"] == MV("n1")  # n1 = n1 self-assignment
    assert cfg["invariants"] == ["LeaderHasAllAckedValues", "NoLogDivergence"]
    assert cfg["view"] == "view" and cfg["symmetry"] == "symmServers"


UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))


@pytest.mark.parametrize("name", sorted(UNSAFE))
def test_unsafe_fixtures_pinned_by_both_oracles(name):
    """Known-unsafe Flexible configs (quorums that do not intersect): the Python
    oracle reproduces the C oracle's violation exactly -- invariant, depth,
    trace length and the counts at the first violating state."""
    g = UNSAFE[name]
    p = bfs(make_spec(g["module"], parse_cfg(g["cfg"])))
    assert (p.status, p.violated, p.depth, len(p.trace)) == (g["status"], g["violated"], g["depth"], g["trace_len"])
    assert (p.generated, p.distinct) == (g["generated"], g["distinct"])


def test_exhausted_rungs_pinned_by_the_c_oracle():
    """The GPU records of the exhaustible BASELINE rungs (tests/golden/
    exhausted.json) equal the C oracle's runs over them level for level --
    the whole rung where the oracle exhausted it (tools/oracle_exhaust.py,
    tools/fold_oracle_rungs.py)."""
    ex = json.load(open(os.path.join(HERE, "golden", "exhausted.json")))
    pinned = 0
    for name, g in ex.items():
        o = g.get("oracle")
        if not o:
            continue
        pinned += 1
        assert o["levels"] == g["levels"][:len(o["levels"])], name
        assert g["oracle_levels"] == len(o["levels"])
        if o["status"] == "ok":
            assert (o["generated"], o["distinct"], o["depth"], o["hidden_same_level"]) == (
                g["generated"], g["distinct"], g["depth"], g["hidden_var_collisions"]), name
            assert len(o["levels"]) == len(g["levels"])
    assert pinned >= 1
