"""The C ABI boundary: librmc.so loads, exports every entry point include/rmc.h
declares, rejects bad input with a message, and fails loudly without a GPU."""
import os
import re

import pytest

import raftmc
from conftest import gpu_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    txt = open(os.path.join(ROOT, "include", "rmc.h")).read()
    return sorted(set(re.findall(r"\b(rmc_[a-z_]+)\s*\(", txt)))


def test_exports_every_declared_symbol():
    L = raftmc.lib()
    names = declared()
    assert set(names) == set(raftmc.EXPORTS)
    for n in names:
        assert hasattr(L, n), n


def test_load_errors_are_reported():
    with pytest.raises(raftmc.RaftmcError, match="unsupported module"):
        raftmc.Model(module="KRaftWithReconfig", cfg_text="CONSTANTS\n")
    with pytest.raises(raftmc.RaftmcError, match="MaxElections"):
        raftmc.Model(module="Raft", cfg_text="CONSTANTS Server = {n1, n2} Value = {v1}\nINIT Init NEXT Next VIEW view")
    with pytest.raises(raftmc.RaftmcError, match="cfg"):
        raftmc.Model(os.path.join(ROOT, "configs", "Raft.tla"), os.path.join(ROOT, "configs", "missing.cfg"))


def test_loads_shipped_cfgs():
    for mod in ("Raft", "PullRaft", "RaftFsync", "FlexibleRaft"):
        raftmc.Model(os.path.join(ROOT, "configs", mod + ".tla"), os.path.join(ROOT, "configs", mod + ".cfg"))


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_check_without_gpu_fails_loudly():
    m = raftmc.Model(os.path.join(ROOT, "configs", "Raft.tla"), os.path.join(ROOT, "configs", "Raft.cfg"))
    with pytest.raises(raftmc.RaftmcError, match="HIP device|no HIP"):
        m.check()
