"""GPU: TLC -dumpTrace for behaviours the HIP search found (SURVEY.md §8f
rank 1).  The error trace of every unsafe fixture is written as a
trace-validation module, replayed by the independent Python oracle's Init and
Next (standing in for TLC, which is absent -- SURVEY.md §8c), and its last
state must violate the reported invariant under the oracle too."""
import json
import os
import subprocess

import pytest

import raftmc
from oracle.pyoracle import make_spec, parse_cfg
from test_trace_module import OracleFormatter, parse_trace_states, replay_with_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
UNSAFE = json.load(open(os.path.join(HERE, "golden", "unsafe.json")))
MEDIUM = json.load(open(os.path.join(HERE, "golden", "medium.json")))
CASES = dict(UNSAFE)
CASES.update({k: v for k, v in MEDIUM.items() if v["status"] == "violation"})

pytestmark = pytest.mark.gpu


def _final_oracle_state(spec, states):
    """Replay (asserting every step) and return the oracle state of the last record."""
    replay_with_oracle(spec, states)
    fmt = OracleFormatter(spec)
    cur = [s for s in spec.init_states() if fmt.state(s) == states[0][1]][0]
    for label, want in states[1:]:
        cur = next(t for name, fn in spec.actions() if name.split("(")[0] == label.split("(")[0]
                   for t in fn(cur) if fmt.state(t) == want)
    return cur


@pytest.mark.parametrize("name", sorted(CASES))
def test_dumped_trace_replays_and_violates(name):
    g = CASES[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    r = m.check()
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    tla, cfg = m.trace_module(g["module"] + "_TTrace")
    states = parse_trace_states(tla)
    assert len(states) == g["trace_len"]
    spec = make_spec(g["module"], parse_cfg(g["cfg"]))
    last = _final_oracle_state(spec, states)
    inv = dict(spec.invariants)[g["violated"]]
    assert not inv(last)
    js = m.trace_json()
    assert len(js["states"]) == g["trace_len"]


def test_cli_dump_trace(tmp_path):
    name = sorted(UNSAFE)[0]
    g = UNSAFE[name]
    cfgp = tmp_path / "Unsafe.cfg"
    cfgp.write_text(g["cfg"])
    out = tmp_path / "Unsafe_TTrace.tla"
    exe = os.path.join(ROOT, "raft-tlaplus_amd", "build", "raftmc")
    p = subprocess.run([exe, "-deadlock", "-config", str(cfgp), "-dumpTrace", "tla", str(out), "-module", g["module"]],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 12, p.stdout + p.stderr  # 12 = invariant violated (TLC's exit code)
    assert "Error: Invariant %s is violated." % g["violated"] in p.stdout
    assert out.exists() and (tmp_path / "Unsafe_TTrace.cfg").exists()
    assert len(parse_trace_states(out.read_text())) == g["trace_len"]
    assert "INIT TraceInit" in (tmp_path / "Unsafe_TTrace.cfg").read_text()
    pj = tmp_path / "t.json"
    p = subprocess.run([exe, "-deadlock", "-config", str(cfgp), "-dumpTrace", "json", str(pj), "-module", g["module"]],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 12
    assert len(json.loads(pj.read_text())["states"]) == g["trace_len"]
