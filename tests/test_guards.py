"""The TLA+ front end's guard compiler (rmc_guard.cpp).

A Next disjunct whose EFFECT is a library action's but whose guard differs --
e.g. Raft.tla:242-257's RequestVote with `electionCtr <= MaxElections` -- is
checked with the library's effect behind its own guard, compiled from TLA+
into the guard machine's code (rmc_spec.h guard_vm) that the kernels and the
CPU engine both run.  CPU tests: (1) every tests/golden/guards.json case, its
guards given as TLA+ text (rmc_model_set_guard), through the CPU engine,
equals the Python oracle with the same guards written in Python
(make_golden.py --guards); (2) the compiler refuses what it cannot compile,
naming it; (3) on the reference module edited in place (skipped where
/root/reference is not mounted) the edited guard is lowered and gives the
same counts, while an edited effect is still refused."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
GUARDS = json.load(open(os.path.join(HERE, "golden", "guards.json")))
REF = "/root/reference/specifications"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")


def model(g):
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    for action, params, expr in g["guards"]:
        m.set_guard(action, params, expr)
    return m


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == (
        g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(GUARDS))
def test_compiled_guards_cpu_engine_equal_oracle(name):
    g = GUARDS[name]
    same(model(g).check_cpu(workers=8, max_depth=g["max_depth"]), g)


def test_guard_changes_the_space():
    """Each case's guard bites: the counts differ from the reference guard's."""
    for name, g in GUARDS.items():
        r = raftmc.Model(module=g["module"], cfg_text=g["cfg"]).check_cpu(workers=8, max_depth=g["max_depth"])
        assert (r["generated"], r["distinct"]) != (g["generated"], g["distinct"]), name


def test_reference_guard_as_text_gives_the_reference_counts():
    """The reference's own RequestVote guard (Raft.tla:243-244), compiled, is
    the built-in guard: same counts as the model without an override."""
    g = GUARDS["raft_rv_le_n2v1e1"]
    base = raftmc.Model(module="Raft", cfg_text=g["cfg"]).check_cpu(workers=4)
    m = raftmc.Model(module="Raft", cfg_text=g["cfg"])
    m.set_guard("RequestVote", "i", "electionCtr < MaxElections /\\ state[i] \\in {Follower, Candidate}")
    r = m.check_cpu(workers=4)
    assert r["levels"] == base["levels"]


def test_set_guard_replaces_an_earlier_guard():
    g = GUARDS["raft_rv_le_n2v1e1"]
    m = raftmc.Model(module="Raft", cfg_text=g["cfg"])
    m.set_guard("RequestVote", "i", "FALSE")
    m.set_guard("RequestVote", "i", g["guards"][0][2])
    same(m.check_cpu(workers=4), g)


@pytest.mark.parametrize("action,params,expr,match", [
    ("RequestVote", "i", "Budget(i)", "Budget"),                                    # unknown operator
    ("RequestVote", "i", "messages = {}", "messages"),                              # a variable it does not read
    ("RequestVote", "i, j", "TRUE", "parameters"),                                  # wrong arity
    ("RequestVote", "i", "state[i] + 1 > 0", "arithmetic"),                         # type error
    ("RequestVote", "i", "\\E j \\in Nat : j > 0", "Server or Value"),              # unbounded set
    ("AppendEntries", "i, j", "TRUE", "not one the front end compiles"),            # a message-carrying action
    ("RequestVote", "i", "1 + (1 + (1 + (1 + (1 + (1 + (1 + (1 + (1 + 1)))))))) > 0", "8-value stack"),
])
def test_guard_compiler_refuses_naming_it(action, params, expr, match):
    m = raftmc.Model(module="Raft", cfg_text=GUARDS["raft_rv_le_n2v1e1"]["cfg"])
    with pytest.raises(raftmc.RaftmcError, match=match):
        m.set_guard(action, params, expr)
    # a refused guard leaves the model as it was
    base = raftmc.Model(module="Raft", cfg_text=GUARDS["raft_rv_le_n2v1e1"]["cfg"]).check_cpu(workers=4)
    assert m.check_cpu(workers=4)["levels"] == base["levels"]


def test_guards_refuse_kraft():
    kr = json.load(open(os.path.join(HERE, "golden", "kraft.json")))
    g = next(iter(kr.values()))
    m = raftmc.Model(module="KRaft", cfg_text=g["cfg"])
    with pytest.raises(raftmc.RaftmcError, match="KRaft"):
        m.set_guard("Restart", "i", "TRUE")


# ---------------------------------------------------------------- reference modules
def ref_text():
    return open(os.path.join(REF, "standard-raft", "Raft.tla")).read()


def load(tmp_path, text, cfg):
    p = tmp_path / "Raft.tla"
    p.write_text(text)
    c = tmp_path / "Raft.cfg"
    c.write_text(cfg)
    return raftmc.Model(str(p), str(c))


@needs_ref
def test_edited_requestvote_guard_is_compiled(tmp_path):
    """Raft.tla:243 edited to `electionCtr <= MaxElections`: lowered onto the
    library's RequestVote effect behind the compiled guard, equal to the
    Python oracle with the same edit."""
    text = ref_text()
    edited = text.replace("    /\\ electionCtr < MaxElections \n", "    /\\ electionCtr <= MaxElections \n")
    assert edited != text
    g = GUARDS["raft_rv_le_n2v1e1"]
    m = load(tmp_path, edited, g["cfg"])
    same(m.check_cpu(workers=8), g)


@needs_ref
def test_edited_becomeleader_guard_is_compiled(tmp_path):
    text = ref_text()
    edited = text.replace("    /\\ votesGranted[i] \\in Quorum\n", "    /\\ votesGranted[i] = Server\n", 1)
    assert edited != text
    g = GUARDS["raft_bl_all_n3v1e1"]
    same(load(tmp_path, edited, g["cfg"]).check_cpu(workers=8), g)


@needs_ref
def test_edited_effect_is_compiled_whole_or_refused(tmp_path):
    """An edited EFFECT is no longer the library's: the action is compiled
    whole (rmc_guard.cpp compile_effect; tests/test_effects.py), so counting
    two elections per RequestVote checks a smaller space; an effect the
    compiler cannot take (electionCtr set from the message bag) is refused
    naming the action."""
    text = ref_text()
    cfg = GUARDS["raft_rv_le_n2v1e1"]["cfg"]
    assert "MaxElections = 1" in cfg
    cfg = cfg.replace("MaxElections = 1", "MaxElections = 2")  # two elections, or one counted twice
    edited = text.replace("    /\\ electionCtr' = electionCtr + 1\n", "    /\\ electionCtr' = electionCtr + 2\n")
    assert edited != text
    m = load(tmp_path, edited, cfg)
    base = raftmc.Model(module="Raft", cfg_text=cfg).check_cpu(workers=4)
    assert m.check_cpu(workers=4)["distinct"] < base["distinct"]
    bad = text.replace("    /\\ electionCtr' = electionCtr + 1\n", "    /\\ electionCtr' = Cardinality(DOMAIN messages)\n")
    assert bad != text
    with pytest.raises(raftmc.RaftmcError, match="RequestVote"):
        load(tmp_path, bad, cfg)
