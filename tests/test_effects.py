"""The TLA+ front end's effect compiler (rmc_guard.cpp
compile_effect): a Next disjunct that matches no library action, neither whole
nor by its effect, is compiled whole -- its guard into the guard machine's
code, its effect (v' = [v EXCEPT ![i] = e] with @, counters, acked, a log
Append, the family's send helpers over RequestVoteRequest records, UNCHANGED)
into the same machine's E_* stores (rmc_spec.h effect_vm) -- and run by the
kernels and the CPU engine alike.

CPU tests: (1) every tests/golden/effects.json case, its actions given as TLA+
text (rmc_model_define_action) and named in Next (rmc_model_set_next),
through the CPU engine, equals the Python oracle with the same actions
written in Python (make_golden.py --effects): counts per level, depth,
status, the violated invariant; (2) a compiled action equal to the
reference's gives the reference's counts; (3) the compiler refuses what it
cannot compile, naming it; (4) on the reference module edited in place
(skipped where /root/reference is not mounted) a new action body is lowered
through the front end and equals the fixture, and a send helper that is not
the family's own is refused."""
import json
import os

import pytest

import raftmc
from cfgs import NEXT_RAFT, cfg_text

HERE = os.path.dirname(os.path.abspath(__file__))
EFFECTS = json.load(open(os.path.join(HERE, "golden", "effects.json")))
REF = "/root/reference/specifications"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")


def model(g):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    for name, form, params, body in g["actions"]:
        m.define_action(name, form, params, body)
    m.set_next(g["next"])
    return m


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (
        g["generated"], g["distinct"], g["depth"], g["status"] if g["status"] != "violation" else "violation")
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]
    if g["status"] == "violation":
        assert r["violated"] == g["violated"]


@pytest.mark.parametrize("name", sorted(EFFECTS))
def test_compiled_actions_cpu_engine_equal_oracle(name):
    g = EFFECTS[name]
    same(model(g).check_cpu(workers=8, max_depth=g["max_depth"]), g)


def test_compiled_actions_change_the_space():
    """Each case's action differs from the library's: the counts differ from
    the module's own Next (same depth bound)."""
    for name, g in EFFECTS.items():
        r = raftmc.Model(module=g["module"], cfg_text=g["cfg"]).check_cpu(workers=8, max_depth=g["max_depth"])
        assert (r["generated"], r["distinct"], r["status"]) != (g["generated"], g["distinct"], g["status"]), name


REFERENCE_RV = """/\\ electionCtr < MaxElections
    /\\ state[i] \\in {Follower, Candidate}
    /\\ state' = [state EXCEPT ![i] = Candidate]
    /\\ currentTerm' = [currentTerm EXCEPT ![i] = currentTerm[i] + 1]
    /\\ votedFor' = [votedFor EXCEPT ![i] = i]
    /\\ votesGranted' = [votesGranted EXCEPT ![i] = {i}]
    /\\ electionCtr' = electionCtr + 1
    /\\ SendMultipleOnce(
           {[mtype         |-> RequestVoteRequest,
             mterm         |-> currentTerm[i] + 1,
             mlastLogTerm  |-> LastTerm(log[i]),
             mlastLogIndex |-> Len(log[i]),
             msource       |-> i,
             mdest         |-> j] : j \\in Server \\ {i}})
    /\\ UNCHANGED <<acked, leaderVars, logVars, restartCtr>>"""


@pytest.mark.parametrize("n,v,E", [(2, 1, 2), (3, 1, 1)])
def test_reference_request_vote_compiled_whole_gives_the_reference_counts(n, v, E):
    """Raft.tla:242-257's RequestVote written out as text and compiled whole
    (guard and effect) checks exactly the built-in lowering's space."""
    cfg = cfg_text("Raft", n=n, v=v, E=E)
    base = raftmc.Model(module="Raft", cfg_text=cfg).check_cpu(workers=8)
    m = raftmc.Model(module="Raft", cfg_text=cfg)
    m.define_action("RequestVoteText", "i", "i", REFERENCE_RV)
    m.set_next(("Restart", "RequestVoteText") + NEXT_RAFT[2:])
    r = m.check_cpu(workers=8)
    assert r["levels"] == base["levels"]
    assert (r["generated"], r["distinct"], r["depth"]) == (base["generated"], base["distinct"], base["depth"])
    assert m.next()[1] == "RequestVoteText"


REFERENCE_BL = """/\\ state[i] = Candidate
    /\\ votesGranted[i] \\in Quorum
    /\\ state'      = [state EXCEPT ![i] = Leader]
    /\\ nextIndex'  = [nextIndex EXCEPT ![i] =
                         [j \\in Server |-> Len(log[i]) + 1]]
    /\\ matchIndex' = [matchIndex EXCEPT ![i] =
                         [j \\in Server |-> 0]]
    /\\ pendingResponse' = [pendingResponse EXCEPT ![i] =
                                [j \\in Server |-> FALSE]]
    /\\ UNCHANGED <<messages, currentTerm, votedFor, candidateVars,
                   auxVars, logVars>>"""
REFERENCE_RESTART = """/\\ restartCtr < MaxRestarts
    /\\ state'           = [state EXCEPT ![i] = Follower]
    /\\ votesGranted'    = [votesGranted EXCEPT ![i] = {}]
    /\\ nextIndex'       = [nextIndex EXCEPT ![i] = [j \\in Server |-> 1]]
    /\\ matchIndex'      = [matchIndex EXCEPT ![i] = [j \\in Server |-> 0]]
    /\\ pendingResponse' = [pendingResponse EXCEPT ![i] = [j \\in Server |-> FALSE]]
    /\\ commitIndex'     = [commitIndex EXCEPT ![i] = 0]
    /\\ restartCtr'      = restartCtr + 1
    /\\ UNCHANGED <<messages, currentTerm, votedFor, log, acked, electionCtr>>"""


@pytest.mark.parametrize("slot,body", [(0, REFERENCE_RESTART), (2, REFERENCE_BL)])
def test_reference_leader_rows_compiled_whole_give_the_reference_counts(slot, body):
    """Raft.tla:226-235's Restart and :289-300's BecomeLeader (the leader's
    rows as [j \\in Server |-> e]) written out and compiled whole check the
    built-in lowering's space."""
    cfg = cfg_text("Raft", n=2, v=1, E=2, R=1)
    base = raftmc.Model(module="Raft", cfg_text=cfg).check_cpu(workers=8)
    m = raftmc.Model(module="Raft", cfg_text=cfg)
    m.define_action("Text", "i", "i", body)
    nxt = list(NEXT_RAFT)
    nxt[slot] = "Text"
    m.set_next(nxt)
    r = m.check_cpu(workers=8)
    assert r["levels"] == base["levels"]
    assert (r["generated"], r["distinct"], r["depth"]) == (base["generated"], base["distinct"], base["depth"])


@pytest.mark.parametrize("body,match", [
    (REFERENCE_RV.replace("UNCHANGED <<acked, leaderVars, logVars, restartCtr>>",
                          "UNCHANGED <<acked, logVars, restartCtr>>"), "Index is neither assigned nor UNCHANGED"),
    (REFERENCE_RV.replace("[votedFor EXCEPT ![i] = i]", "[votedFor EXCEPT ![j] = i]"), "own server"),
    (REFERENCE_RV.replace("/\\ electionCtr' = electionCtr + 1", "/\\ nextIndex' = nextIndex")
     .replace("leaderVars, ", "matchIndex, pendingResponse, electionCtr, "), "nextIndex"),
    (REFERENCE_RV.replace("mtype         |-> RequestVoteRequest", "mtype         |-> AppendEntriesRequest"),
     "RequestVoteRequest records only"),
    (REFERENCE_RV.replace("/\\ electionCtr' = electionCtr + 1", "/\\ electionCtr' = electionCtr + 1\n"
                          "    /\\ electionCtr' = electionCtr + 2"), "changed twice"),
    (REFERENCE_RV.replace("[state EXCEPT ![i] = Candidate]", "[state EXCEPT ![i] = 3]"), "integer"),
    # {rec : j \in S} with records that need not differ per member
    # (TLC's set would hold one where one send per member would add two)
    (REFERENCE_RV.replace("mdest         |-> j] : j", "mdest         |-> i] : j"), "mdest is not j"),
])
def test_refused_effects_are_named(body, match):
    m = raftmc.Model(module="Raft", cfg_text=cfg_text("Raft", n=2, v=1, E=1))
    with pytest.raises(raftmc.RaftmcError, match=match):
        m.define_action("Bad", "i", "i", body)


def test_define_action_is_refused_for_other_families():
    m = raftmc.Model(module="PullRaft", cfg_text=cfg_text("PullRaft", n=2, v=1, E=1))
    with pytest.raises(raftmc.RaftmcError, match="Raft, FlexibleRaft and RaftFsync"):
        m.define_action("X", "i", "i", REFERENCE_RV)


def _edited_raft(old, new):
    text = open(os.path.join(REF, "standard-raft", "Raft.tla")).read()
    assert old in text
    return text.replace(old, new, 1)


@needs_ref
def test_module_with_a_new_action_body_equals_the_fixture(tmp_path):
    """Raft.tla with RequestVote's self vote taken out (votedFor' = Nil,
    votesGranted' = {}): the front end compiles the edited action whole, and
    the check equals the Python oracle's fixture for the same edit."""
    g = EFFECTS["raft_rv_noself_n3v1e2"]
    text = _edited_raft("/\\ votedFor' = [votedFor EXCEPT ![i] = i]", "/\\ votedFor' = [votedFor EXCEPT ![i] = Nil]")
    old = "/\\ votesGranted'   = [votesGranted EXCEPT ![i] = {i}]"  # Raft.tla:248's own spacing
    assert old in text
    text = text.replace(old, "/\\ votesGranted' = [votesGranted EXCEPT ![i] = {}]", 1)
    (tmp_path / "Raft.tla").write_text(text)
    (tmp_path / "Raft.cfg").write_text(g["cfg"])
    m = raftmc.Model(tla_path=str(tmp_path / "Raft.tla"))
    assert m.next()[1] == "RequestVote"  # the module's own name, compiled whole
    same(m.check_cpu(workers=8, max_depth=g["max_depth"]), g)


@needs_ref
def test_module_send_helper_must_be_the_familys_own(tmp_path):
    """A RequestVote whose SendMultipleOnce is redefined (here: to send with
    count 2) is not the family's helper: refused, naming it."""
    g = EFFECTS["raft_rv_noself_n3v1e2"]
    text = _edited_raft("/\\ votedFor' = [votedFor EXCEPT ![i] = i]", "/\\ votedFor' = [votedFor EXCEPT ![i] = Nil]")
    old = "messages' = messages @@ [msg \\in msgs |-> 1]"
    assert old in text
    text = text.replace(old, "messages' = messages @@ [msg \\in msgs |-> 2]")
    (tmp_path / "Raft.tla").write_text(text)
    (tmp_path / "Raft.cfg").write_text(g["cfg"])
    with pytest.raises(raftmc.RaftmcError, match="SendMultipleOnce"):
        raftmc.Model(tla_path=str(tmp_path / "Raft.tla"))
