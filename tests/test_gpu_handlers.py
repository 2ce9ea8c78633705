"""GPU: message handlers compiled whole by the TLA+ front end (rmc_guard.cpp
compile_handler) checked by the kernels: k_expand evaluates every compiled
handler on every DOMAIN element in phase B (its own ordinal range, its binding
nfixed + 128 (1 + q) + k), phase C and k_materialize re-run the same program.
Every case equals the Python oracle's fixture (tests/golden/handlers.json) in
one chunk, in 37-parent chunks, on two logical shards, on two threads of the
in-process multi-GPU driver, with the host frontier, and a violation's trace
is rebuilt through the compiled handler.
"""
import json
import os

import pytest

import raftmc
from cfgs import HANDLERS

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "handlers.json")))
CASES = {h[0]: h for h in HANDLERS}

pytestmark = pytest.mark.gpu


def model(name):
    _, module, kw, nxt, acts, md = CASES[name]
    m = raftmc.Model(module=module, cfg_text=FIX[name]["cfg"])
    for a, form, params, body in acts:
        m.define_action(a, form, params, body)
    m.set_next(list(nxt))
    return m


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["status"] == g["status"]
    if g["status"] == "ok":
        assert r["levels"] == g["levels"]
        assert r["hidden_var_collisions"] == g["hidden_same_level"]
    else:
        assert r["violated"] == g["violated"]
        assert len(r["trace"]) == g["trace_len"]


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("how", ["one", "chunks37", "shards2", "threads2", "hostfrontier"])
def test_gpu_matches_oracle(name, how):
    m = model(name)
    md = CASES[name][5]
    if how == "one":
        r = m.check(max_depth=md)
    elif how == "chunks37":
        r = m.check(chunk_parents=37, max_depth=md)
    elif how == "shards2":
        r = m.check_logical(2, chunk_parents=101, max_depth=md)
    elif how == "threads2":
        r = m.check_multi([0, 0], chunk_parents=101, max_depth=md)
    else:
        r = m.check(host_frontier=1, chunk_parents=53, max_depth=md)
    same(r, FIX[name])


def test_gpu_trace_equals_cpu_engine():
    name = "flex_hrvresp_all_n2v1e2"
    g = model(name).check()
    c = model(name).check_cpu(workers=4)
    assert g["status"] == "violation" and g["trace"] == c["trace"]
    assert "HRVRespAll" in [a for a, _ in g["trace"]]


def test_gpu_fresh_model_widens_with_handlers():
    """Rows start at N message slots and widen mid-check: the compiled
    handlers' bindings do not depend on the slot count."""
    m = model("raft_rejae_lenidx_n2v2e2")
    same(m.check(chunk_parents=29), FIX["raft_rejae_lenidx_n2v2e2"])
    assert m.selftest_widenings()


def test_gpu_simulate_with_a_compiled_handler():
    """Simulation draws among every enabled binding, the compiled handlers' included."""
    r = model("flex_hrvresp_all_n2v1e2").simulate(walkers=4096, depth=40, seed=7)
    assert r["status"] in ("ok", "violation")
    if r["status"] == "violation":
        assert r["violated"] == "LeaderHasAllAckedValues"
