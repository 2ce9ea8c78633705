"""PullRaftVariant2 (pull-raft/PullRaftVariant2.tla) on
the CPU: both oracles on the committed fixtures (tests/golden/variant2.json,
made by `make_golden.py --variant2`), the lowered actions replayed on the host
(rmc_spec.h, the code the kernels run) and the CPU engine (same layout and
first-in-TLC-order rule as the GPU path).  The shipped cfg's fixture is in
shipped.json (C oracle): 1,454,442 distinct, 891 same-level hidden-variable
collisions (2,615 when the last successor in TLC order wins instead)."""
import json
import os

import pytest

import raftmc
from oracle import run_c
from oracle.pyoracle import make_spec
from oracle.pyoracle.cfg import parse_cfg
from oracle.pyoracle.tlc import bfs

HERE = os.path.dirname(os.path.abspath(__file__))
V2 = json.load(open(os.path.join(HERE, "golden", "variant2.json")))
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))
FAST = sorted(k for k in V2 if V2[k]["distinct"] <= 10000 and "_n5" not in k)


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", FAST)
def test_python_oracle_reproduces_fixture(name):
    g = V2[name]
    p = bfs(make_spec(g["module"], parse_cfg(g["cfg"])))
    assert (p.generated, p.distinct, p.depth, [list(x) for x in p.levels], p.hidden_same_level) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"], g["hidden_same_level"])


@pytest.mark.parametrize("name", sorted(V2))
def test_c_oracle_reproduces_fixture(name):
    g = V2[name]
    cfg = parse_cfg(g["cfg"])
    c = run_c.run(g["module"], cfg["constants"], cfg["invariants"], threads=4)
    assert (c["generated"], c["distinct"], c["depth"], c["levels"], c["hidden_same_level"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"], g["hidden_same_level"])


@pytest.mark.parametrize("name", FAST)
def test_host_replay_of_lowered_actions(name):
    g = V2[name]
    r = raftmc.Model(module=g["module"], cfg_text=g["cfg"]).selftest_host_bfs()
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]


def test_host_replay_n5_prefix():
    """5 servers (120 permutations, votesLastEntry relabelled): first levels on the host."""
    g = V2["pull2_n5v1e1"]
    r = raftmc.Model(module=g["module"], cfg_text=g["cfg"]).selftest_host_bfs(max_distinct=2000)
    n = len(r["levels"])
    assert n >= 10 and r["levels"] == g["levels"][:n]


@pytest.mark.parametrize("name", sorted(V2))
@pytest.mark.parametrize("workers,chunk", [(8, 0), (3, 97)])
def test_cpu_engine(name, workers, chunk):
    g = V2[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_cpu(workers=workers, chunk_parents=chunk), g)


def test_cpu_engine_shipped_cfg_first_wins():
    """The shipped cfg: TLC-order winners decide the hidden-variable collision
    count (891; the reverse-order probe counts 2,615)."""
    g = SHIPPED["PullRaftVariant2_cfg"]
    ROOT = os.path.dirname(HERE)
    m = raftmc.Model(module="PullRaftVariant2", cfg_path=os.path.join(ROOT, g["cfg_path"]))
    r = m.check_cpu(workers=8)
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
        (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert r["hidden_var_collisions"] == g["hidden_same_level"] == 891


def test_fixtures_exercise_the_variant2_actions():
    """Truncation on a failed pull and LeaderNotify with a last common entry occur."""
    g = V2["pull2_n3v1e2"]["action_counts"]
    assert g["HandleFailPullEntriesResponse"] > 0 and g["LearnOfLeader"] > 0 and g["RejectPullEntriesRequest"] > 0
