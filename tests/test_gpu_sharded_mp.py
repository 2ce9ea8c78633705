"""GPU: the fingerprint-sharded protocol (raft-tlaplus_amd/csrc/rmc_sharded.cpp)
run by SEVERAL PROCESSES, one shard each, as on a multi-GPU node -- here all on
one GPU, with shared memory as the transport (rmc_check_sharded_shm) because
RCCL refuses two ranks per device.  Every rank must report the oracle's global
result.  (The gloo test, tests/test_sharded_gloo.py, runs a Python restatement
of the protocol; this runs the product's own C++.)"""
import json
import os
import subprocess
import sys
import uuid

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


def run_ranks(world, fx, key, chunk=0, extra=(), env_of=None):
    """env_of(rank) -> extra environment variables for that rank's process."""
    name = "rmc_test_" + uuid.uuid4().hex[:12]
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "sharded_shm_rank.py"), str(r), str(world), name,
                               fx, key, str(chunk)] + [str(x) for x in extra], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=dict(os.environ, **(env_of(r) if env_of else {})))
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            tails = [q.communicate()[1][-1500:] for q in procs]
            raise AssertionError("ranks hung; stderr tails:\n" + "\n----\n".join(tails))
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    return outs


@pytest.mark.parametrize("world,fx,key,chunk", [
    (2, "small.json", "raft_n3v1e1", 0),
    (3, "small.json", "pull_n3v2e1", 97),
    (2, "variant2.json", "pull2_n3v2e1", 0),
    (4, "kraft.json", "kraft_n3v2e1", 1000),
    (2, "small.json", "raft_n2v2e2", 7),
    (5, "small.json", "raft_n3v1e1", 33),
    (2, "shipped.json", "Raft_cfg", 100000),   # Raft.cfg: 8,664,032 distinct, levels of up to 10 rounds
    (3, "shipped.json", "PullRaftVariant2_cfg", 0),  # 891 same-level hidden-variable collisions
])
def test_multiprocess_shards_match_oracle(world, fx, key, chunk):
    g = json.load(open(os.path.join(HERE, "golden", fx)))[key]
    for r in run_ranks(world, fx, key, chunk):
        assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
            (g["generated"], g["distinct"], g["depth"], g["status"])
        assert r["levels"] == g["levels"]
        assert r["hidden_var_collisions"] == g["hidden_same_level"]


def test_multiprocess_shards_violation():
    g = json.load(open(os.path.join(HERE, "golden", "kraft.json")))["kraft_n3v1e1r1"]
    for r in run_ranks(2, "kraft.json", "kraft_n3v1e1r1"):
        assert r["status"] == "violation" and r["violated"] == g["violated"] and r["depth"] == g["depth"]
        # TLC's counts at the failing state, summed over the ranks' blocks of the round
        assert (r["generated"], r["distinct"]) == (g["generated"], g["distinct"])


def test_one_rank_out_of_host_pages_stops_every_rank():
    """host pages are per process, so one rank runs out first.  Its
    failure is agreed through the next allgather instead of leaving its peers
    in a collective: rank 1 gets a host-page limit far below the shipped
    Raft.cfg's levels (1000-row pages), rank 0 none -- both ranks end with
    status "capacity" and the same completed levels, a prefix of the fixture's."""
    g = json.load(open(os.path.join(HERE, "golden", "shipped.json")))["Raft_cfg"]
    env = lambda r: {"RMC_HOST_PAGE_ROWS": "1000", **({"RMC_HOST_FRONTIER_GIB": "0.01"} if r == 1 else {})}
    outs = run_ranks(2, "shipped.json", "Raft_cfg", 20000, extra=(1,), env_of=env)
    assert [o["status"] for o in outs] == ["capacity", "capacity"], outs
    assert "host frontier pages exhausted" in outs[1]["message"]
    assert "another rank" in outs[0]["message"]
    k = len(outs[0]["levels"])
    assert outs[1]["levels"] == outs[0]["levels"] == g["levels"][:k] and 2 < k < len(g["levels"])
