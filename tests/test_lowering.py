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
