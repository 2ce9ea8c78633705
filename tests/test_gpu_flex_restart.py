"""GPU parity for FlexibleRaft's Restart (FlexibleRaft.tla:200-208: a server
restarts as a Follower keeping currentTerm, votedFor and log, its volatile
state reset) with MaxRestarts >= 1 (tests/golden/flex_restart.json, cfgs.py
FLEX_RESTART): every level, the hidden-variable collisions (restartCtr is
hidden by the VIEW), the invariants' outcome, through the single-shard search,
small chunks, 2 logical shards and the host frontier."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
FR = json.load(open(os.path.join(HERE, "golden", "flex_restart.json")))
CASES = sorted(FR)

pytestmark = pytest.mark.gpu


def run(g, how):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    depth = 0 if g["status"] != "truncated" else g["depth"]
    if how == "single":
        return m.check(max_depth=depth)
    if how == "chunks":
        return m.check(max_depth=depth, chunk_parents=777)
    if how == "shards2":
        return m.check_logical(2, max_depth=depth)
    return m.check(max_depth=depth, host_frontier=1, chunk_parents=5000)


@pytest.mark.parametrize("how", ["single", "chunks", "shards2", "host"])
@pytest.mark.parametrize("name", CASES)
def test_flex_restart_matches_oracle(name, how):
    g = FR[name]
    r = run(g, how)
    if g["status"] == "violation":
        assert r["status"] == "violation" and r["violated"] == g["violated"]
        assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
        assert len(r["trace"]) == g["trace_len"]
        return
    assert r["levels"] == g["levels"]
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["status"] == ("ok" if g["status"] == "ok" else "stopped")
    assert r["hidden_var_collisions"] == g["hidden_same_level"]
