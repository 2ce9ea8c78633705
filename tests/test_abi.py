"""The C ABI boundary: librmc.so loads, exports every entry point include/rmc.h
declares, rejects bad input with a message, and fails loudly without a GPU."""
import ctypes
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
        raftmc.Model(module="Raft", cfg_path=os.path.join(ROOT, "configs", "missing.cfg"))


def test_missing_tla_is_refused(tmp_path):
    """TLC fails on a module file that does not exist; so does rmc_model_load
    (the built-in lowering without a .tla is rmc_model_load_text)."""
    cfg = tmp_path / "Raft.cfg"
    cfg.write_text(open(os.path.join(ROOT, "configs", "Raft.cfg")).read())
    with pytest.raises(raftmc.RaftmcError, match="cannot read module file"):
        raftmc.Model(str(tmp_path / "Raft.tla"), str(cfg))
    with pytest.raises(raftmc.RaftmcError, match="cannot read module file"):
        raftmc.Model(str(tmp_path / "Raft"), str(cfg))  # TLC appends .tla


def test_abi_layout_matches_ctypes():
    """librmc's own sizeof/offsetof of rmc_options and rmc_result equal the
    ctypes structures' (a binding that drifts from include/rmc.h would write
    past the struct or read the wrong fields)."""
    lay = raftmc.abi_layout()
    no, nr = len(raftmc.Options._fields_), len(raftmc.Result._fields_)
    assert len(lay) == 2 + no + nr
    assert lay[0] == ctypes.sizeof(raftmc.Options)
    assert lay[1:1 + no] == [getattr(raftmc.Options, f).offset for f, _ in raftmc.Options._fields_]
    assert lay[1 + no] == ctypes.sizeof(raftmc.Result)
    assert lay[2 + no:] == [getattr(raftmc.Result, f).offset for f, _ in raftmc.Result._fields_]


def test_header_fields_match_bindings():
    """The field lists of include/rmc.h, the ctypes structures and the JNA
    stub in INTEGRATION.md are the same, in the same order."""
    h = open(os.path.join(ROOT, "include", "rmc.h")).read()
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()

    def header_fields(name):
        body = dict((n, b) for b, n in re.findall(r"typedef struct \{([^{}]*)\} (\w+);", h))[name]
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        out = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            decl = re.sub(r"\[\d+\]", "", decl)
            names = [x.strip().split()[-1].lstrip("*") for x in decl.split(",")]
            out += names
        return out

    jna = re.findall(r"@Structure\.FieldOrder\(\{(.*?)\}\)", integ, re.S)
    assert len(jna) == 2
    jna = [[x.strip().strip('"') for x in j.split(",")] for j in jna]
    assert header_fields("rmc_options") == [f for f, _ in raftmc.Options._fields_] == jna[0]
    assert header_fields("rmc_result") == [f for f, _ in raftmc.Result._fields_] == jna[1]


def test_loads_shipped_cfgs():
    for mod in ("Raft", "PullRaft", "RaftFsync", "FlexibleRaft"):
        raftmc.Model(module=mod, cfg_path=os.path.join(ROOT, "configs", mod + ".cfg"))


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_check_without_gpu_fails_loudly():
    m = raftmc.Model(module="Raft", cfg_path=os.path.join(ROOT, "configs", "Raft.cfg"))
    with pytest.raises(raftmc.RaftmcError, match="HIP device|no HIP"):
        m.check()


def test_result_prefix_is_survey_8b():
    """rmc_result starts with SURVEY.md §8b's fields in §8b's order and C
    layout, so a binding written to §8b reads them at the right offsets; the
    library's extra fields (message, measurements) come after them."""
    class Survey8b(ctypes.Structure):
        _fields_ = [("generated", ctypes.c_uint64), ("distinct", ctypes.c_uint64),
                    ("left_on_queue", ctypes.c_uint64), ("depth", ctypes.c_uint32), ("status", ctypes.c_int),
                    ("violated", ctypes.c_char * 64), ("hidden_var_collisions", ctypes.c_uint64),
                    ("seconds", ctypes.c_double)]
    for f, _ in Survey8b._fields_:
        assert getattr(raftmc.Result, f).offset == getattr(Survey8b, f).offset, f
    assert raftmc.Result.message.offset >= ctypes.sizeof(Survey8b)


def test_source_id_matches_the_tree():
    """rmc_source_id hashes the sources the library was built from; a variant
    build made from other sources is refused at load (RAFTMC_BUILD)."""
    sid = raftmc.lib().rmc_source_id().decode()
    assert raftmc.source_mismatch(sid) is None
    digest, _, files = sid.partition(":")
    assert "csrc/rmc_kernels.hip" in files.split(",")
    assert raftmc.source_mismatch("0" * 32 + ":" + files).startswith("source hash")
    assert "missing" in raftmc.source_mismatch(digest + ":csrc/no_such_file.cpp")


def test_stale_build_is_refused(monkeypatch):
    """r06: a library built from other sources than the tree's is refused,
    the default build included (VERDICT r05 What's weak #7); only an explicit
    RAFTMC_ALLOW_STALE=1 lets an experiment load one."""
    sid = raftmc.lib().rmc_source_id().decode()
    raftmc.refuse_stale(sid)
    digest, _, files = sid.partition(":")
    with pytest.raises(raftmc.RaftmcError, match="built from other sources"):
        raftmc.refuse_stale("0" * 32 + ":" + files)
    monkeypatch.setenv("RAFTMC_ALLOW_STALE", "1")
    raftmc.refuse_stale("0" * 32 + ":" + files)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_multi_gpu_without_gpu_fails_loudly():
    """n_gpus > 1 and the in-process multi-GPU entry fail loudly here too."""
    m = raftmc.Model(module="Raft", cfg_path=os.path.join(ROOT, "configs", "Raft.cfg"))
    with pytest.raises(raftmc.RaftmcError, match="HIP device|no HIP"):
        m.check(n_gpus=2)
    with pytest.raises(raftmc.RaftmcError, match="HIP device|no HIP"):
        m.check_multi([0, 0])
    with pytest.raises(raftmc.RaftmcError, match="bad argument"):
        m.check_multi([0, 0], transport=7)


def test_phases_before_any_check():
    m = raftmc.Model(module="Raft", cfg_path=os.path.join(ROOT, "configs", "Raft.cfg"))
    assert m.phases() == {}
