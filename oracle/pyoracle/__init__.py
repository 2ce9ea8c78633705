"""Python oracle: literal restatements of the four Raft specs under TLC semantics.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import this package, and only as the
checker.  The product path (raft-tlaplus_amd/) never imports it.

Parity unpinned against TLC: the reference holds no counts, traces or
fixtures and TLC (Java) is absent here and on the GPU box.
The pins are the hand-derived first levels of SURVEY.md Appendix B and the
agreement of this oracle with the independent C oracle (oracle/cengine).
"""
from .cfg import load_cfg, parse_cfg
from .tlc import bfs, EvalError


def make_spec(module, cfg, next_order=None, guards=None, defined=None):
    from .raft import RaftSpec
    from .variants import FlexibleRaftSpec, RaftFsyncSpec, PullRaftSpec, PullRaftVariant2Spec
    from .kraft import KRaftSpec
    table = {"Raft": RaftSpec, "FlexibleRaft": FlexibleRaftSpec,
             "RaftFsync": RaftFsyncSpec, "PullRaft": PullRaftSpec,
             "PullRaftVariant2": PullRaftVariant2Spec, "KRaft": KRaftSpec}
    if module not in table:
        raise ValueError("oracle: unsupported module %r" % module)
    kw = {}
    if next_order:
        kw["next_order"] = next_order
    if guards:
        if module == "KRaft":
            raise ValueError("oracle: guard overrides are not offered for KRaft")
        kw["guards"] = guards
    if defined:
        if module not in ("Raft", "FlexibleRaft", "RaftFsync"):
            raise ValueError("oracle: defined actions are offered for Raft, FlexibleRaft and RaftFsync")
        kw["defined"] = defined
    return table[module](cfg["constants"], invariants=tuple(cfg["invariants"]), **kw)
