"""The lowered actions (rmc_spec.h, the code the kernels run) executed on the
host through librmc's test hook, against the oracle fixtures.  CPU only; this
is not a product path (rmc_check never reaches it)."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))


@pytest.mark.parametrize("name", sorted(SMALL))
def test_host_replay_of_lowered_actions(name):
    g = SMALL[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.selftest_host_bfs()
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["levels"] == g["levels"]


N5 = json.load(open(os.path.join(HERE, "golden", "n5.json")))


@pytest.mark.parametrize("name", sorted(k for k in N5 if N5[k]["status"] in ("ok", "truncated")))
def test_host_replay_n5_prefix(name):
    """5 servers (120 permutations): the lowered actions and the signature-pruned
    canonical fingerprint reproduce the oracle's first levels on the host."""
    g = N5[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.selftest_host_bfs(max_distinct=20000)
    n = len(r["levels"])
    assert n >= 10 and r["levels"] == g["levels"][:n]
