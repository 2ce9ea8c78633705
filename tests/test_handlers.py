"""CPU: message handlers compiled whole by the TLA+ front end (rmc_guard.cpp
compile_handler).

A Next disjunct `\\E m \\in DOMAIN messages : body` whose text differs from every
lowered handler is compiled into one effect_vm program: its guards read the
bound message's fields and messages[m], its effects act on m.mdest, Discard(m)
and Reply(record, m) update the bag.  tests/golden/handlers.json holds the
Python oracle's counts for the same handlers written in Python
(make_golden.py --handlers); the CPU engine runs the same compiled code as the
kernels.  The GPU side is tests/test_gpu_handlers.py.
"""
import json
import os

import pytest

import raftmc
from cfgs import HANDLERS, cfg_text

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "handlers.json")))
CASES = {h[0]: h for h in HANDLERS}
REF = "/root/reference/specifications"


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


def test_fixture_set_matches_cfgs():
    assert set(FIX) == set(CASES)


@pytest.mark.parametrize("name", sorted(CASES))
def test_cpu_engine_matches_oracle(name):
    same(model(name).check_cpu(workers=8, max_depth=CASES[name][5]), FIX[name])


@pytest.mark.parametrize("name", ["raft_hrvresp_text_n3v1e1", "raft_rejae_text_n2v2e2", "fsync_rejae_text_n2v1e2r1",
                                  "raft_haeresp_text_n3v1e1", "fsync_haeresp_text_n2v1e2r1"])
def test_reference_text_compiled_gives_the_builtin_space(name):
    """The reference's HandleRequestVoteResponse (Raft.tla:386-401),
    RejectAppendEntriesRequest (:412-430, RaftFsync.tla's) and
    HandleAppendEntriesResponse (:490-505, RaftFsync.tla:486-500) written out
    and compiled whole check exactly the library handler's space, level by
    level."""
    _, module, kw, nxt, acts, md = CASES[name]
    base = raftmc.Model(module=module, cfg_text=FIX[name]["cfg"]).check_cpu(workers=8)
    r = model(name).check_cpu(workers=8)
    assert r["levels"] == base["levels"]
    assert (r["generated"], r["distinct"], r["depth"], r["hidden_var_collisions"]) == \
        (base["generated"], base["distinct"], base["depth"], base["hidden_var_collisions"])


def test_violation_trace_names_the_compiled_handler():
    g = FIX["flex_hrvresp_all_n2v1e2"]
    r = model("flex_hrvresp_all_n2v1e2").check_cpu(workers=4)
    assert r["status"] == "violation" and r["violated"] == g["violated"]
    labels = [a for a, _ in r["trace"]]
    assert labels[0] == "Initial predicate"
    assert "HRVRespAll" in labels


def test_two_handlers_keep_their_order():
    """Two compiled handlers in one Next: each has its own ordinal range (its
    DOMAIN elements in TLC order), so the hidden-variable collisions and the
    per-level counts equal the oracle's."""
    same(model("raft_two_handlers_n2v1e2r1").check_cpu(workers=8), FIX["raft_two_handlers_n2v1e2r1"])


def _cfg():
    return cfg_text("Raft", n=2, v=1, E=1)


@pytest.mark.parametrize("body,match", [
    # an effect at the message's source, not its destination
    ("""/\\ ReceivableMessage(m, RequestVoteResponse, EqualTerm)
    /\\ votesGranted' = [votesGranted EXCEPT ![m.msource] = {}]
    /\\ Discard(m)
    /\\ UNCHANGED <<serverVars, leaderVars, logVars, auxVars>>""", "own server"),
    # a disjunction of effects whose guards may both hold
    ("""/\\ ReceivableMessage(m, RequestVoteResponse, EqualTerm)
    /\\ \\/ /\\ m.mvoteGranted
          /\\ votesGranted' = [votesGranted EXCEPT ![m.mdest] = {}]
       \\/ /\\ m.mterm > 0
          /\\ UNCHANGED votesGranted
    /\\ Discard(m)
    /\\ UNCHANGED <<serverVars, leaderVars, logVars, auxVars>>""", "complementary"),
    # a reply of a request record
    ("""/\\ ReceivableMessage(m, RequestVoteResponse, EqualTerm)
    /\\ Reply([mtype |-> RequestVoteRequest, mterm |-> 1, mlastLogTerm |-> 0, mlastLogIndex |-> 0,
              msource |-> m.mdest, mdest |-> m.msource], m)
    /\\ UNCHANGED <<serverVars, candidateVars, leaderVars, logVars, auxVars>>""", "replies with"),
    # the message itself as a value
    ("""/\\ m = m
    /\\ Discard(m)
    /\\ UNCHANGED <<serverVars, candidateVars, leaderVars, logVars, auxVars>>""", "itself as a value"),
    # a field the records do not have
    ("""/\\ m.mnothing = 1
    /\\ Discard(m)
    /\\ UNCHANGED <<serverVars, candidateVars, leaderVars, logVars, auxVars>>""", "no field mnothing"),
    # a variable left undetermined
    ("""/\\ ReceivableMessage(m, RequestVoteResponse, EqualTerm)
    /\\ Discard(m)
    /\\ UNCHANGED <<serverVars, leaderVars, logVars, auxVars>>""", "votesGranted is neither"),
])
def test_refused_handlers_are_named(body, match):
    m = raftmc.Model(module="Raft", cfg_text=_cfg())
    with pytest.raises(raftmc.RaftmcError, match=match):
        m.define_action("Bad", "m", "m", body)


def test_min_max_of_a_literal_only():
    """Min / Max (Raft.tla:190-192) of a one- or two-element literal compile to
    a compare and select; of any other set they are refused."""
    m = raftmc.Model(module="Raft", cfg_text=_cfg())
    with pytest.raises(raftmc.RaftmcError, match="literal of one or two integers"):
        m.define_action("Bad", "m", "m", """/\\ ReceivableMessage(m, AppendEntriesResponse, EqualTerm)
    /\\ nextIndex' = [nextIndex EXCEPT ![m.mdest][m.msource] = Max({k \\in 1..3 : k > 1})]
    /\\ Discard(m)
    /\\ UNCHANGED <<serverVars, candidateVars, matchIndex, pendingResponse, logVars, auxVars>>""")
    # a guard through the same code: Min of two terms, Max of one
    g = raftmc.Model(module="Raft", cfg_text=_cfg())
    g.set_guard("RequestVote", "i", "Min({currentTerm[i], 1}) = 0 /\\ Max({electionCtr}) < MaxElections")
    base = raftmc.Model(module="Raft", cfg_text=_cfg())
    base.set_guard("RequestVote", "i", "currentTerm[i] = 0 /\\ electionCtr < MaxElections")
    assert g.check_cpu(workers=4)["levels"] == base.check_cpu(workers=4)["levels"]


def test_discard_outside_a_handler_is_refused():
    m = raftmc.Model(module="Raft", cfg_text=_cfg())
    with pytest.raises(raftmc.RaftmcError, match="changes nothing|Discard|message"):
        m.define_action("Bad", "i", "i", """/\\ state[i] = Leader
    /\\ Discard(i)
    /\\ UNCHANGED <<serverVars, candidateVars, leaderVars, logVars, auxVars>>""")


def test_handlers_are_refused_for_other_families():
    m = raftmc.Model(module="PullRaft", cfg_text=cfg_text("PullRaft", n=2, v=1, E=1))
    with pytest.raises(raftmc.RaftmcError, match="Raft, FlexibleRaft and RaftFsync"):
        m.define_action("X", "m", "m", "/\\ messages[m] > 0\n    /\\ UNCHANGED <<messages>>")


@pytest.mark.skipif(not os.path.isdir(REF), reason="edits the reference module text (build container only)")
def test_module_with_an_edited_handler_loads_through_the_front_end(tmp_path):
    """Raft.tla with HandleRequestVoteResponse tallying every response (its
    mvoteGranted test dropped) is lowered with that handler compiled whole and
    equals the fixture -- the .tla path of define_action."""
    text = open(os.path.join(REF, "standard-raft", "Raft.tla")).read()
    a = text.index("HandleRequestVoteResponse ==")
    b = text.index("RejectAppendEntriesRequest ==", a)
    b = text.rindex("\\* ACTION", a, b)
    edited = text[:a] + "HandleRequestVoteResponse ==\n    \\E m \\in DOMAIN messages :\n        " + \
        CASES["raft_hrvresp_all_n2v1e2"][4][0][3].replace("\n", "\n    ") + "\n\n" + text[b:]
    (tmp_path / "Raft.tla").write_text(edited)
    (tmp_path / "Raft.cfg").write_text(FIX["raft_hrvresp_all_n2v1e2"]["cfg"])
    m = raftmc.Model(str(tmp_path / "Raft.tla"), str(tmp_path / "Raft.cfg"))
    assert "HandleRequestVoteResponse" in m.next()
    same(m.check_cpu(workers=8), FIX["raft_hrvresp_all_n2v1e2"])
