"""TLC -dumpTrace: the trace-validation module and the
JSON trace librmc writes for an error behaviour, checked on the CPU.

TLC is not available here or on the GPU box, so the module's
claim -- TraceStates is a behaviour of the spec, replayed by its own Init and
Next -- is checked with the independent Python oracle standing in for TLC's
evaluation of TraceInit/TraceNext: the first record must be the oracle's
initial state and every next record one of the oracle's successors of the
previous one, with the same action name.  The behaviours are seeded random
walks over librmc's lowered actions (test hook rmc_selftest_random_trace),
replayed into the model's trace exactly as after a violation.
"""
import json
import os
import re

import pytest

import raftmc
from oracle.pyoracle import make_spec, parse_cfg
from oracle.pyoracle.tlc import NIL, Rec

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))


def _squash(text):
    return re.sub(r"\s+", "", text)


class OracleFormatter:
    """Oracle states -> TLC value text (the syntax of TLC's error traces)."""

    def __init__(self, spec):
        self.spec = spec
        self.sn = spec.server_names
        self.vn = spec.value_names

    def srv(self, i):
        return "Nil" if i == NIL else self.sn[i]

    def val(self, x):
        if isinstance(x, bool):
            return "TRUE" if x else "FALSE"
        return str(x)

    def rec(self, r, field_fmt):
        return "[" + ", ".join("%s |-> %s" % (k, field_fmt(k, v)) for k, v in tuple.__iter__(r)) + "]"

    def entry(self, e):
        return "[term |-> %d, value |-> %s]" % (e.term, self.vn[e.value])

    def msg_field(self, k, v):
        if k in ("mdest", "msource"):
            return self.srv(v)
        if k == "mentries":
            return "<<" + ", ".join(self.entry(e) for e in v) + ">>"
        if k == "mlastCommonEntry":
            return self.rec(v, lambda kk, vv: str(vv))
        return self.val(v)

    def fn(self, xs, f):
        return "(" + " @@ ".join("%s :> %s" % (self.sn[i], f(x)) for i, x in enumerate(xs)) + ")"

    def var(self, name, x):
        if name == "messages":
            if not x:
                return "<< >>"
            return "(" + " @@ ".join("%s :> %d" % (self.rec(m, self.msg_field), c) for m, c in x) + ")"
        if name == "acked":
            return "(" + " @@ ".join("%s :> %s" % (self.vn[v], "Nil" if a == NIL else self.val(a))
                                     for v, a in enumerate(x)) + ")"
        if name in ("electionCtr", "restartCtr"):
            return str(x)
        if name in ("votedFor", "leader"):
            return self.fn(x, self.srv)
        if name == "log":
            return self.fn(x, lambda lg: "<<" + ", ".join(self.entry(e) for e in lg) + ">>")
        if name == "votesGranted":
            return self.fn(x, lambda s: "{" + ", ".join(self.sn[j] for j in sorted(s)) + "}")
        if name in ("nextIndex", "matchIndex", "pendingResponse"):
            return self.fn(x, lambda row: self.fn(row, self.val))
        return self.fn(x, self.val)  # currentTerm, state, commitIndex, fsyncIndex

    def state(self, s):
        return {v: _squash(self.var(v, s[v])) for v in self.spec.variables}


def parse_trace_states(module_text):
    """[(action label, {var: squashed value text})] from TraceStates == << ... >>."""
    body = module_text.split("TraceStates == <<\n", 1)[1].split("\n>>\n", 1)[0]
    parts = re.split(r"  \\\* State (\d+): (.*)\n  \[", body)
    out = []
    for k in range(1, len(parts), 3):
        assert int(parts[k]) == len(out) + 1
        label, rec = parts[k + 1], parts[k + 2].rstrip().rstrip(",")
        assert rec.endswith("]")
        fields = {}
        for f in rec[:-1].split(",\n   "):
            var, val = f.split(" |-> ", 1)
            fields[var] = _squash(val)
        out.append((label, fields))
    return out


def replay_with_oracle(spec, states):
    """Check states[0] is an initial state and each step a Next step (TLC's TraceNext)."""
    fmt = OracleFormatter(spec)
    inits = [s for s in spec.init_states() if fmt.state(s) == states[0][1]]
    assert inits, "TraceStates[1] is not an initial state of the spec"
    cur = inits[0]
    actions = spec.actions()
    for k in range(1, len(states)):
        label, want = states[k]
        nxt = None
        for name, fn in actions:
            if name.split("(")[0] != label.split("(")[0]:
                continue
            for t in fn(cur):
                if fmt.state(t) == want:
                    nxt = t
                    break
            if nxt is not None:
                break
        assert nxt is not None, "step %d (%s) is not a Next step of the spec" % (k + 1, label)
        cur = nxt


@pytest.mark.parametrize("name", sorted(SMALL))
@pytest.mark.parametrize("seed", [1, 2])
def test_trace_module_replays_under_oracle_next(name, seed):
    g = SMALL[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    n = m.selftest_random_trace(seed, 40)
    assert n >= 2
    tla, cfg = m.trace_module(g["module"] + "_TTrace")
    # module shape: header, EXTENDS the checked spec, one record per state,
    # TraceInit/TraceNext over every variable, the acceptance invariant
    assert tla.startswith("-" * 28 + " MODULE %s_TTrace " % g["module"])
    assert "EXTENDS %s, Sequences, TLC\n" % g["module"] in tla
    assert tla.rstrip().endswith("=" * 77)
    assert "TraceAccepted == traceIdx < Len(TraceStates)" in tla
    spec = make_spec(g["module"], parse_cfg(g["cfg"]))
    for v in spec.variables:
        assert "/\\ %s = TraceStates[1].%s" % (v, v) in tla
        assert "/\\ %s' = TraceStates[traceIdx + 1].%s" % (v, v) in tla
    states = parse_trace_states(tla)
    assert len(states) == n
    assert [list(s[1]) for s in states] == [list(spec.variables)] * n
    # the records are the same states rmc_trace_state prints in TLC's error trace
    tr = m.trace()
    for (label, fields), (act, text) in zip(states, tr):
        printed = {ln.split(" = ", 1)[0][3:]: _squash(ln.split(" = ", 1)[1])
                   for ln in re.split(r"\n(?=/\\ )", text.strip())}
        assert printed == fields
    replay_with_oracle(spec, states)
    # companion cfg: the model's constants, the trace spec, the acceptance invariant
    assert "INIT TraceInit\nNEXT TraceNext\nINVARIANT TraceAccepted\n" in cfg
    for sname in spec.server_names:
        assert "    %s = %s\n" % (sname, sname) in cfg
    # JSON form of the same behaviour
    js = m.trace_json()
    assert js["module"] == g["module"] and len(js["states"]) == n
    assert js["states"][0]["action"] == "Initial predicate"
    for st, (_, fields) in zip(js["states"], states):
        assert {v: _squash(st[v]) for v in spec.variables} == fields
