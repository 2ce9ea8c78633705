"""GPU: the classic Raft safety properties as opt-in invariants
(ElectionSafety, LogMatching, LeaderCompleteness, StateMachineSafety --
north_star's in-kernel invariant checks; the reference's cfgs check only
LeaderHasAllAckedValues and NoLogDivergence).  Fixtures
(tests/golden/extras.json): both oracles agree on the counts, the violated
invariant and the trace length; the k_materialize invariant pass must too,
single-shard, with small chunks and with 2 logical shards, and a violation's
trace must replay in the oracle and end in a state violating it there."""
import json
import os

import pytest

import raftmc
from oracle.pyoracle import make_spec, parse_cfg
from test_gpu_trace import _final_oracle_state
from test_trace_module import parse_trace_states

HERE = os.path.dirname(os.path.abspath(__file__))
EXTRAS = json.load(open(os.path.join(HERE, "golden", "extras.json")))

pytestmark = pytest.mark.gpu


def run(g, how):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    if how == "single":
        return m, m.check()
    if how == "chunks":
        return m, m.check(chunk_parents=7)
    return m, m.check_logical(2)


@pytest.mark.parametrize("how", ["single", "chunks", "shards2"])
@pytest.mark.parametrize("name", sorted(EXTRAS))
def test_classic_invariants_match_oracle(name, how):
    g = EXTRAS[name]
    m, r = run(g, how)
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    if g["status"] != "violation":
        assert r["levels"] == g["levels"]
        return
    assert r["violated"] == g["violated"] and len(r["trace"]) == g["trace_len"]
    tla, _ = m.trace_module(g["module"] + "_TTrace")
    spec = make_spec(g["module"], parse_cfg(g["cfg"]))
    last = _final_oracle_state(spec, parse_trace_states(tla))
    assert not dict(spec.invariants)[g["violated"]](last)
