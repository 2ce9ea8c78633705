"""The drop-in boundary on the reference's own files (CPU): TLC's contract is
`tlc2.TLC -deadlock -config M.cfg M.tla`, so rmc_model_load must accept the
reference's .tla/.cfg texts verbatim (cfg quirks included: `n1 = n1`
self-assignments, Raft.cfg:6-9; `v2` used undeclared, PullRaft.cfg:11), and
must refuse a .tla whose definitions differ from the spec it lowers (instead
of silently checking the built-in lowering).  Skipped where the reference is
not mounted (it never is on the GPU box)."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/specifications"
SPECS = {"Raft": "standard-raft", "FlexibleRaft": "flexible-raft", "PullRaft": "pull-raft",
         "RaftFsync": "raft-and-fsync", "PullRaftVariant2": "pull-raft", "KRaft": "pull-raft"}
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")


def ref(module, ext):
    return os.path.join(REF, SPECS[module], module + ext)


@pytest.mark.parametrize("module", sorted(SPECS))
def test_reference_files_load_verbatim(module):
    m = raftmc.Model(ref(module, ".tla"), ref(module, ".cfg"))
    assert m is not None


@pytest.mark.parametrize("name", sorted(SHIPPED))
def test_reference_cfg_same_first_levels(name):
    """The reference cfg text, loaded verbatim, gives the oracle's first levels
    (through the CPU engine: same lowering as the GPU path)."""
    g = SHIPPED[name]
    m = raftmc.Model(ref(g["module"], ".tla"), ref(g["module"], ".cfg"))
    r = m.check_cpu(workers=8, max_depth=14)
    assert r["levels"] == g["levels"][:14]


def test_edited_spec_is_not_checked_as_the_built_in_one(tmp_path):
    """Raft with an action whose EFFECT computes something else (Restart
    counting two restarts, Raft.tla:234) is a different spec: never checked
    as the built-in one.  The front end compiles that action whole
    (rmc_guard.cpp compile_effect; its counts against the Python oracle:
    tests/test_effects.py), and an effect it cannot compile -- here an
    AppendEntries request sent by Restart -- is refused naming the action.
    (An edited GUARD is compiled behind the library's effect:
    tests/test_guards.py; re-enabling the commented-out DuplicateMessage
    disjunct, Raft.tla:540, is lowered: tests/test_frontend.py.)"""
    txt = open(ref("Raft", ".tla")).read()
    edited = txt.replace("    /\\ restartCtr'      = restartCtr + 1\n", "    /\\ restartCtr'      = restartCtr + 2\n")
    assert edited != txt
    p = tmp_path / "Raft.tla"
    p.write_text(edited)
    m = raftmc.Model(str(p), ref("Raft", ".cfg"))
    builtin = raftmc.Model(module="Raft", cfg_path=ref("Raft", ".cfg"))
    assert m.next() == builtin.next()  # the module's own names; Restart now compiled whole
    bad = txt.replace("    /\\ restartCtr'      = restartCtr + 1\n",
                      "    /\\ restartCtr'      = restartCtr + 1\n    /\\ Send([mtype |-> AppendEntriesRequest])\n")
    bad = bad.replace("UNCHANGED <<messages, currentTerm, votedFor, log, acked, electionCtr>>",
                      "UNCHANGED <<currentTerm, votedFor, log, acked, electionCtr>>", 1)
    assert bad != txt
    p.write_text(bad)
    with pytest.raises(raftmc.RaftmcError, match="Restart"):
        raftmc.Model(str(p), ref("Raft", ".cfg"))


def test_edited_guard_is_lowered(tmp_path):
    """Restart gated on restartCtr <= MaxRestarts instead of < (Raft.tla:227):
    the library's Restart effect behind the compiled guard (rmc_guard.cpp)."""
    txt = open(ref("Raft", ".tla")).read()
    edited = txt.replace("    /\\ restartCtr < MaxRestarts\n", "    /\\ restartCtr <= MaxRestarts\n")
    assert edited != txt
    p = tmp_path / "Raft.tla"
    p.write_text(edited)
    m = raftmc.Model(str(p), ref("Raft", ".cfg"))
    assert m.next() == raftmc.Model(module="Raft", cfg_path=ref("Raft", ".cfg")).next()


def test_comment_and_layout_edits_pass(tmp_path):
    txt = open(ref("Raft", ".tla")).read()
    p = tmp_path / "Raft.tla"
    p.write_text("\\* a local note\n" + txt.replace("\n\n", "\n  \n").replace("Init ==", "Init  =="))
    raftmc.Model(str(p), ref("Raft", ".cfg"))


def test_classic_invariants_unknown_on_the_tla_path(tmp_path):
    """TLC resolves INVARIANT names in the module; the reference Raft.tla does
    not define ElectionSafety, so on the TLC-compatible path (a .tla given) the
    name is refused as undefined -- the built-in extras are available only
    through rmc_model_load_text / raftmc -module."""
    cfg = open(ref("Raft", ".cfg")).read().replace("NoLogDivergence", "NoLogDivergence\n    ElectionSafety")
    p = tmp_path / "Raft.cfg"
    p.write_text(cfg)
    with pytest.raises(raftmc.RaftmcError, match="not defined in module Raft"):
        raftmc.Model(ref("Raft", ".tla"), str(p))
    raftmc.Model(module="Raft", cfg_text=cfg)  # the extras path
