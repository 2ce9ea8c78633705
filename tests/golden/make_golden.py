"""Generate the committed golden fixtures (tests/golden/*.json).

Run in the build container (needs oracle/_build/rmc_oracle: `make -C oracle`):
    python tests/golden/make_golden.py [--shipped]

Every SMALL case is computed twice, by the literal Python oracle and by the
C oracle, and written only if the two agree on generated/distinct/depth and
every per-level count.  --shipped adds the shipped reference configs (C oracle
only; minutes of CPU).  The reference itself records no counts anywhere
(SURVEY.md §4, §8c): these vectors are pinned by the hand-derived first levels
of SURVEY.md Appendix B plus the agreement of two independent restatements.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import run_c  # noqa: E402
from oracle.pyoracle import make_spec  # noqa: E402
from oracle.pyoracle.cfg import parse_cfg  # noqa: E402
from oracle.pyoracle.tlc import bfs  # noqa: E402
from cfgs import (EFFECTS, EXTRAS, HANDLERS, FLEX_RESTART, FRONTEND, GUARDS, LADDERS, MEDIUM, N5, N5_UNSAFE, ORDER, SMALL, UNSAFE, VARIANT2_MEDIUM,  # noqa: E402
                  VARIANT2_N5, VARIANT2_SMALL, cfg_text)

SHIPPED = [  # the reference's own cfgs, restated in configs/ (same constants)
    ("Raft_cfg", "Raft", "configs/Raft.cfg"),
    ("PullRaft_cfg", "PullRaft", "configs/PullRaft.cfg"),
    ("RaftFsync_cfg", "RaftFsync", "configs/RaftFsync.cfg"),
    ("PullRaftVariant2_cfg", "PullRaftVariant2", "configs/PullRaftVariant2.cfg"),
]


def unsafe():
    """--unsafe: known-unsafe configs, C oracle with the violating trace's length."""
    out = {}
    for name, module, kw in UNSAFE:
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=1, extra=["--trace"])
        out[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], violated=c["violated"], trace_len=len(c.get("trace", [])),
                         pinned_by="coracle")
        print(name, c["generated"], c["distinct"], c["depth"], c["status"], c["violated"], flush=True)
    with open(os.path.join(HERE, "unsafe.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def n5():
    """--n5: 5-server cases, level-truncated (cfgs.N5).  The C oracle runs to the
    first level boundary past max_distinct; the Python oracle runs a shorter
    prefix and must agree with the C oracle on every level it completed."""
    only_unsafe = "--n5-unsafe" in sys.argv
    out = json.load(open(os.path.join(HERE, "n5.json"))) if only_unsafe else {}
    for name, module, kw, c_max, py_max in ([] if only_unsafe else N5):
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=8,
                      extra=["--max-distinct", str(c_max)])
        p = bfs(make_spec(module, cfg), max_states=py_max)
        pl = [list(x) for x in p.levels]
        if pl != c["levels"][:len(pl)]:
            raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pl, c["levels"][:len(pl)]))
        out[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"],
                         depth=c["depth"], status=c["status"], levels=c["levels"], max_distinct=c_max,
                         max_msgs=c["max_msgs"], hidden_same_level=c["hidden_same_level"],
                         pyoracle_levels=len(pl), pinned_by="coracle; first %d levels pyoracle==coracle" % len(pl))
        print(name, c["generated"], c["distinct"], c["depth"], "py levels", len(pl), flush=True)
    for name, module, kw in N5_UNSAFE:  # C oracle only (the Python oracle would take hours)
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=1, extra=["--trace"])
        out[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], violated=c["violated"], levels=c["levels"],
                         trace_len=len(c.get("trace", [])), pinned_by="coracle")
        print(name, c["generated"], c["distinct"], c["depth"], c["status"], c["violated"], flush=True)
    with open(os.path.join(HERE, "n5.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def order():
    """--order: TLC-order first-wins fixtures (cfgs.ORDER).  Both oracles where the
    Python one finishes in minutes; the C oracle's --reverse-order counts are
    recorded beside them (different counts = the winner choice matters)."""
    out = {}
    for name, module, kw in ORDER:
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=4)
        rv = run_c.run(module, cfg["constants"], cfg["invariants"], threads=1, extra=["--reverse-order"])
        pinned = "coracle"
        if c["distinct"] <= 400000:
            p = bfs(make_spec(module, cfg))
            pr = (p.generated, p.distinct, p.depth, p.status, [list(x) for x in p.levels], p.hidden_same_level)
            cr = (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"], c["hidden_same_level"])
            if pr != cr:
                raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pr[:4] + pr[5:], cr[:4] + cr[5:]))
            pinned = "pyoracle==coracle"
        out[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], levels=c["levels"], max_msgs=c["max_msgs"],
                         hidden_same_level=c["hidden_same_level"], hidden_cross_level=c["hidden_cross_level"],
                         reverse_order=dict(generated=rv["generated"], distinct=rv["distinct"]), pinned_by=pinned)
        print(name, c["generated"], c["distinct"], c["hidden_same_level"], "reverse:", rv["generated"], rv["distinct"],
              pinned, flush=True)
    with open(os.path.join(HERE, "order.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def variant2():
    """--variant2: PullRaftVariant2 fixtures (tests/golden/variant2.json): small
    cases by both oracles (every level, hidden collisions), medium by the C
    oracle, the 5-server case level-truncated (both oracles on the prefix the
    Python one completes), each with the C oracle's --reverse-order counts."""
    M = "PullRaftVariant2"
    out = {}
    for name, kw in VARIANT2_SMALL:
        txt = cfg_text(M, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(M, cfg["constants"], cfg["invariants"], threads=4)
        p = bfs(make_spec(M, cfg))
        pr = (p.generated, p.distinct, p.depth, p.status, [list(x) for x in p.levels], p.hidden_same_level)
        cr = (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"], c["hidden_same_level"])
        if pr != cr:
            raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pr[:4], cr[:4]))
        out[name] = dict(module=M, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], levels=c["levels"], action_counts=c["action_counts"],
                         max_msgs=c["max_msgs"], hidden_same_level=c["hidden_same_level"],
                         pinned_by="pyoracle==coracle")
        print(name, c["generated"], c["distinct"], c["depth"], flush=True)
    for name, kw in VARIANT2_MEDIUM:
        txt = cfg_text(M, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(M, cfg["constants"], cfg["invariants"], threads=8)
        out[name] = dict(module=M, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], levels=c["levels"], action_counts=c["action_counts"],
                         max_msgs=c["max_msgs"], hidden_same_level=c["hidden_same_level"], pinned_by="coracle")
        print(name, c["generated"], c["distinct"], c["depth"], flush=True)
    for name, kw, c_max, py_max in VARIANT2_N5:
        txt = cfg_text(M, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(M, cfg["constants"], cfg["invariants"], threads=8, extra=["--max-distinct", str(c_max)])
        p = bfs(make_spec(M, cfg), max_states=py_max)
        pl = [list(x) for x in p.levels]
        if pl != c["levels"][:len(pl)]:
            raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pl, c["levels"][:len(pl)]))
        out[name] = dict(module=M, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], levels=c["levels"], max_distinct=c_max, max_msgs=c["max_msgs"],
                         hidden_same_level=c["hidden_same_level"], pyoracle_levels=len(pl),
                         pinned_by="coracle; first %d levels pyoracle==coracle" % len(pl))
        print(name, c["generated"], c["distinct"], c["depth"], "py levels", len(pl), flush=True)
    for name, g in out.items():
        if g["status"] != "ok":
            continue
        cfg = parse_cfg(g["cfg"])
        rv = run_c.run(M, cfg["constants"], cfg["invariants"], threads=1, extra=["--reverse-order"])
        g["reverse_order"] = dict(generated=rv["generated"], distinct=rv["distinct"])
    with open(os.path.join(HERE, "variant2.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def ladders():
    """--ladders: BASELINE configs 2 and 5 at their scaled bounds (cfgs.LADDERS),
    level-truncated: the C oracle to the first level boundary past max_distinct,
    the Python oracle on a shorter prefix that must agree level by level."""
    only = sys.argv[sys.argv.index("--ladder-one") + 1] if "--ladder-one" in sys.argv else None
    lp = os.path.join(HERE, "ladders.json")
    out = json.load(open(lp)) if only and os.path.exists(lp) else {}
    for name, module, path, c_max, py_max in LADDERS:
        if only and name != only:
            continue
        with open(os.path.join(ROOT, path)) as fh:
            txt = fh.read()
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=8, extra=["--max-distinct", str(c_max)])
        p = bfs(make_spec(module, cfg), max_states=py_max)
        pl = [list(x) for x in p.levels]
        if pl != c["levels"][:len(pl)]:
            raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pl, c["levels"][:len(pl)]))
        out[name] = dict(module=module, cfg_path=path, generated=c["generated"], distinct=c["distinct"],
                         depth=c["depth"], status=c["status"], levels=c["levels"], max_distinct=c_max,
                         max_msgs=c["max_msgs"], hidden_same_level=c["hidden_same_level"], pyoracle_levels=len(pl),
                         pinned_by="coracle; first %d levels pyoracle==coracle" % len(pl),
                         oracle_seconds=c["seconds"])
        print(name, c["generated"], c["distinct"], c["depth"], "py levels", len(pl), flush=True)
    with open(os.path.join(HERE, "ladders.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def flex_restart():
    """--flex-restart: FlexibleRaft with MaxRestarts >= 1 (cfgs.FLEX_RESTART;
    FlexibleRaft.tla:200-208).  Exhaustive cases: both oracles on every level
    (the Python one on a prefix where it would take too long); the 5-server
    case level-truncated like --n5."""
    M = "FlexibleRaft"
    out = {}
    for name, kw, c_max, py_max in FLEX_RESTART:
        txt = cfg_text(M, **kw)
        cfg = parse_cfg(txt)
        extra = ["--max-distinct", str(c_max)] if c_max else []
        c = run_c.run(M, cfg["constants"], cfg["invariants"], threads=8, extra=extra + ["--trace"])
        p = bfs(make_spec(M, cfg), max_states=py_max) if py_max else bfs(make_spec(M, cfg))
        pl = [list(x) for x in p.levels]
        if py_max:
            if pl != c["levels"][:len(pl)]:
                raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pl, c["levels"][:len(pl)]))
            pinned = "coracle; first %d levels pyoracle==coracle" % len(pl)
        else:
            pr = (p.generated, p.distinct, p.depth, p.status, pl, p.hidden_same_level)
            cr = (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"], c["hidden_same_level"])
            if pr != cr:
                raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pr[:4], cr[:4]))
            pinned = "pyoracle==coracle"
        out[name] = dict(module=M, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], violated=c["violated"], levels=c["levels"],
                         action_counts=c["action_counts"], max_msgs=c["max_msgs"],
                         hidden_same_level=c["hidden_same_level"], trace_len=len(c.get("trace", [])),
                         pyoracle_levels=len(pl), pinned_by=pinned)
        if c_max:
            out[name]["max_distinct"] = c_max
        print(name, c["generated"], c["distinct"], c["depth"], c["status"], c["violated"], pinned, flush=True)
    with open(os.path.join(HERE, "flex_restart.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def extras():
    """--extras: the opt-in classic invariants (cfgs.EXTRAS) -- both oracles must
    agree on the counts and on which invariant fails (and the trace length)."""
    out = {}
    for name, module, kw, inv in EXTRAS:
        txt = cfg_text(module, inv=inv, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=4, extra=["--trace"])
        p = bfs(make_spec(module, cfg))
        pr = (p.generated, p.distinct, p.depth, p.status, [list(x) for x in p.levels])
        cr = (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"])
        if pr != cr or (c["status"] == "violation" and p.violated != c["violated"]):
            raise SystemExit("oracles disagree on %s: py=%s %s c=%s %s" % (name, pr[:4], getattr(p, "violated", ""),
                                                                          cr[:4], c["violated"]))
        out[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"], depth=c["depth"],
                         status=c["status"], violated=c["violated"], levels=c["levels"],
                         hidden_same_level=c["hidden_same_level"], trace_len=len(c.get("trace", [])),
                         pinned_by="pyoracle==coracle")
        print(name, c["generated"], c["distinct"], c["depth"], c["status"], c["violated"], flush=True)
    with open(os.path.join(HERE, "extras.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def frontend():
    """--frontend: modules whose Next the TLA+ front end lowers differently from
    the reference's (cfgs.FRONTEND), by the Python oracle with the same Next
    (every level, hidden-variable collisions; max_depth-truncated where
    DuplicateMessage makes the space infinite).  The C oracle has no
    configurable Next, so these are pinned by the Python oracle alone."""
    out = {}
    for name, module, kw, nxt, md in FRONTEND:
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        p = bfs(make_spec(module, cfg, next_order=nxt), max_depth=md or None)
        out[name] = dict(module=module, cfg=txt, next=list(nxt), max_depth=md, generated=p.generated,
                         distinct=p.distinct, depth=p.depth, status=p.status, levels=[list(x) for x in p.levels],
                         hidden_same_level=p.hidden_same_level, max_msgs=p.max_msgs, pinned_by="pyoracle")
        print(name, p.generated, p.distinct, p.depth, p.status, p.hidden_same_level, "%.1fs" % p.seconds, flush=True)
    with open(os.path.join(HERE, "frontend.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def _guard_py():
    """The Python side of every cfgs.GUARDS guard: {case: {action: g(spec, s, *args)}}."""
    from oracle.pyoracle.raft import CANDIDATE, FOLLOWER, LEADER
    from oracle.pyoracle.tlc import NIL
    st, term = (lambda s, i: s["state"][i]), (lambda s, i: s["currentTerm"][i])

    def quant_rv(sp, s, i):
        busy = any(st(s, j) == LEADER for j in sp.Server)
        return (s["electionCtr"] < sp.MaxElections and st(s, i) in (FOLLOWER, CANDIDATE) and
                (len([j for j in sp.Server if term(s, j) > term(s, i)]) > 0 if busy else True))
    return {
        "raft_rv_le_n2v1e1": {"RequestVote": lambda sp, s, i: s["electionCtr"] <= sp.MaxElections and
                              st(s, i) in (FOLLOWER, CANDIDATE)},
        "raft_bl_all_n3v1e1": {"BecomeLeader": lambda sp, s, i: st(s, i) == CANDIDATE and
                               s["votesGranted"][i] == frozenset(sp.Server)},
        "raft_restart_nonleader_n2v1e2r1": {"Restart": lambda sp, s, i: s["restartCtr"] < sp.MaxRestarts and
                                            st(s, i) != LEADER},
        "raft_client_lastterm_n2v2e2": {"ClientRequest": lambda sp, s, i, v: st(s, i) == LEADER and
                                        s["acked"][v] == NIL and sp.LastTerm(s["log"][i]) < term(s, i)},
        "raft_quant_n2v1e2": {"BecomeLeader": lambda sp, s, i: st(s, i) == CANDIDATE and
                              sp.IsQuorum(s["votesGranted"][i]) and all(term(s, j) <= term(s, i) for j in sp.Server),
                              "RequestVote": quant_rv},
        "flex_bl_card_n3v1e1": {"BecomeLeader": lambda sp, s, i: st(s, i) == CANDIDATE and
                                len(s["votesGranted"][i]) >= 3},
        "fsync_timeout_rvij_n2v1e2r1": {"Timeout": lambda sp, s, i: s["electionCtr"] < sp.MaxElections and
                                        st(s, i) == FOLLOWER,
                                        "RequestVote": lambda sp, s, i, j: st(s, i) == CANDIDATE and i != j and
                                        term(s, j) <= term(s, i)},
        "pull_rv_noleader_n2v1e2r1": {"RequestVote": lambda sp, s, i: s["electionCtr"] < sp.MaxElections and
                                    st(s, i) in (FOLLOWER, CANDIDATE) and s["leader"][i] == NIL},
        "pull2_restart_emptylog_n2v1e2r1": {"Restart": lambda sp, s, i: s["restartCtr"] < sp.MaxRestarts and
                                            len(s["log"][i]) == 0},
    }


def guards():
    """--guards: actions behind a guard other than the reference's (cfgs.GUARDS),
    by the Python oracle with the same guard (_guard_py, written here by hand
    from each TLA+ guard).  The C oracle has no configurable guards, so these
    are pinned by the Python oracle alone."""
    py = _guard_py()
    out = {}
    for name, module, kw, gs, md in GUARDS:
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        p = bfs(make_spec(module, cfg, guards=py[name]), max_depth=md or None)
        out[name] = dict(module=module, cfg=txt, guards=[list(g) for g in gs], max_depth=md, generated=p.generated,
                         distinct=p.distinct, depth=p.depth, status=p.status, levels=[list(x) for x in p.levels],
                         hidden_same_level=p.hidden_same_level, max_msgs=p.max_msgs, pinned_by="pyoracle")
        print(name, p.generated, p.distinct, p.depth, p.status, p.hidden_same_level, "%.1fs" % p.seconds, flush=True)
    with open(os.path.join(HERE, "guards.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def _effect_py():
    """The Python side of every cfgs.EFFECTS action (written here by hand from
    each TLA+ body): {case: {name: (form, f(spec, s, *args))}}."""
    from oracle.pyoracle.raft import CANDIDATE, FOLLOWER, LEADER, RVREQ
    from oracle.pyoracle.tlc import NIL, Rec, fset, fset2

    def rv(spec, s, i, self_vote, step, mstep=None):
        # RequestVote (Raft.tla:242-257) with the self vote optional, a term step
        # and the requests' term step
        if not (s["electionCtr"] < spec.MaxElections and s["state"][i] in (FOLLOWER, CANDIDATE)):
            return
        term = s["currentTerm"][i] + step
        ms = [Rec(mtype=RVREQ, mterm=s["currentTerm"][i] + (step if mstep is None else mstep), mlastLogTerm=spec.LastTerm(s["log"][i]), mlastLogIndex=len(s["log"][i]),
                  msource=i, mdest=j) for j in spec.Server if j != i]
        msgs = spec.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, CANDIDATE)
        t["currentTerm"] = fset(s["currentTerm"], i, term)
        t["votedFor"] = fset(s["votedFor"], i, i if self_vote else NIL)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset([i]) if self_vote else frozenset())
        t["electionCtr"] = s["electionCtr"] + 1
        t["messages"] = msgs
        yield t

    def client_eager(spec, s, i, v):
        if not (s["state"][i] == LEADER and s["acked"][v] == NIL):
            return
        t = dict(s)
        t["log"] = fset(s["log"], i, s["log"][i] + (Rec(term=s["currentTerm"][i], value=v),))
        t["acked"] = fset(s["acked"], v, True)
        yield t

    def restart_keep(spec, s, i):
        if not s["restartCtr"] < spec.MaxRestarts:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 1
        yield t

    def resend(spec, s, i, j, empty):
        # one RequestVoteRequest by the family's Send (Raft: count + 1; RaftFsync: once)
        if not (s["state"][i] == CANDIDATE and i != j):
            return
        m = Rec(mtype=RVREQ, mterm=s["currentTerm"][i], mlastLogTerm=0 if empty else spec.LastTerm(s["log"][i]),
                mlastLogIndex=0 if empty else len(s["log"][i]), msource=i, mdest=j)
        msgs = spec.Send(s["messages"], m)
        if msgs is None:
            return
        t = dict(s)
        t["messages"] = msgs
        yield t

    def restart_two(spec, s, i):
        if not s["restartCtr"] < spec.MaxRestarts:
            return
        N = spec.N
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        t["pendingResponse"] = fset(s["pendingResponse"], i, tuple(False for _ in range(N)))
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 2
        yield t

    def bl_next1(spec, s, i):
        if not (s["state"][i] == CANDIDATE and spec.IsQuorum(s["votesGranted"][i])):
            return
        N = spec.N
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(len(s["log"][i]) if j == i else 0 for j in range(N)))
        row = list(s["pendingResponse"][i])
        row[i] = True
        t["pendingResponse"] = fset(s["pendingResponse"], i, tuple(row))
        yield t

    return {
        "raft_restart_two_n2v1e2r3": {"RestartTwo": ("i", restart_two)},
        "raft_bl_next1_n2v1e2": {"BecomeLeaderNext1": ("i", bl_next1)},
        "raft_rv_noself_n3v1e2": {"RequestVoteNoSelf": ("i", lambda sp, s, i: rv(sp, s, i, False, 1))},
        "raft_rv_term2_n2v1e2": {"RequestVoteTwo": ("i", lambda sp, s, i: rv(sp, s, i, True, 2, 1))},
        "raft_client_eager_n3v1e2": {"ClientRequestEager": ("iv", client_eager)},
        "raft_restart_keep_n2v1e2r1": {"RestartKeep": ("i", restart_keep)},
        "raft_resend_rv_n2v1e1": {"ResendVote": ("ij", lambda sp, s, i, j: resend(sp, s, i, j, False))},
        "fsync_rvij_empty_n2v1e2r1": {"RequestVoteEmpty": ("ij", lambda sp, s, i, j: resend(sp, s, i, j, True))},
        "flex_rv_noself_n3v1e1": {"RequestVoteNoSelf": ("i", lambda sp, s, i: rv(sp, s, i, False, 1))},
    }


def effects():
    """--effects: Next with actions the front end compiles whole (cfgs.EFFECTS),
    by the Python oracle with the same actions written in Python (_effect_py).
    The C oracle has no configurable actions, so these are pinned by the Python
    oracle alone."""
    py = _effect_py()
    path = os.path.join(HERE, "effects.json")
    only = [a.split("=", 1)[1].split(",") for a in sys.argv if a.startswith("--only=")]
    out = json.load(open(path)) if only and os.path.exists(path) else {}
    for name, module, kw, nxt, acts, md in EFFECTS:
        if only and name not in only[0]:
            continue
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        p = bfs(make_spec(module, cfg, next_order=nxt, defined=py[name]), max_depth=md or None)
        out[name] = dict(module=module, cfg=txt, next=list(nxt), actions=[list(a) for a in acts], max_depth=md,
                         generated=p.generated, distinct=p.distinct, depth=p.depth, status=p.status,
                         violated=getattr(p, "violated", None), levels=[list(x) for x in p.levels],
                         hidden_same_level=p.hidden_same_level, max_msgs=p.max_msgs, pinned_by="pyoracle")
        print(name, p.generated, p.distinct, p.depth, p.status, getattr(p, "violated", None), p.hidden_same_level,
              "%.1fs" % p.seconds, flush=True)
    out = {k: v for k, v in out.items() if k in {e[0] for e in EFFECTS}}
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def _handler_py():
    """The Python side of every cfgs.HANDLERS message handler (written here by
    hand from each TLA+ body, iterating DOMAIN messages in TLC's order as the
    oracle's own handlers do): {case: {name: ("m", f(spec, s))}}."""
    from oracle.pyoracle.raft import AEREQ, AERESP, EQUAL, FOLLOWER, LEQ, RVREQ, RVRESP
    from oracle.pyoracle.tlc import NIL, Rec, fset, fset2

    def hrvresp_all(sp, s):
        for m, c in s["messages"]:
            if not sp.ReceivableMessage(s, m, c, RVRESP, EQUAL):
                continue
            i, j = m.mdest, m.msource
            msgs = sp.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            t["votesGranted"] = fset(s["votesGranted"], i, s["votesGranted"][i] | {j})
            t["messages"] = msgs
            yield t

    def hrvreq_nolog(sp, s):
        for m, c in s["messages"]:
            if not sp.ReceivableMessage(s, m, c, RVREQ, LEQ):
                continue
            i, j = m.mdest, m.msource
            grant = m.mterm == s["currentTerm"][i] and s["votedFor"][i] in (NIL, j)
            if not m.mterm <= s["currentTerm"][i]:
                continue
            msgs = sp.Reply(s["messages"], Rec(mtype=RVRESP, mterm=s["currentTerm"][i], mvoteGranted=grant,
                                               msource=i, mdest=j), m)
            if msgs is None:
                continue
            t = dict(s)
            if grant:
                t["votedFor"] = fset(s["votedFor"], i, j)
            t["messages"] = msgs
            yield t

    def rejae_lenidx(sp, s):
        for m, c in s["messages"]:
            if not sp.ReceivableMessage(s, m, c, AEREQ, LEQ):
                continue
            i, j = m.mdest, m.msource
            cur = s["currentTerm"][i]
            if not (m.mterm < cur or (m.mterm == cur and s["state"][i] == FOLLOWER and not sp.LogOk(s, i, m))):
                continue
            msgs = sp.Reply(s["messages"], Rec(mtype=AERESP, mterm=cur, msuccess=False,
                                               mmatchIndex=len(s["log"][i]), msource=i, mdest=j), m)
            if msgs is None:
                continue
            t = dict(s)
            t["messages"] = msgs
            yield t

    def updateterm_stay(sp, s):
        for m, _ in s["messages"]:
            d = m.mdest
            if m.mterm > s["currentTerm"][d]:
                t = dict(s)
                t["currentTerm"] = fset(s["currentTerm"], d, m.mterm)
                t["votedFor"] = fset(s["votedFor"], d, NIL)
                yield t

    def haeresp_resend(sp, s):
        for m, c in s["messages"]:
            if not sp.ReceivableMessage(s, m, c, AERESP, EQUAL):
                continue
            i, j = m.mdest, m.msource
            msgs = sp.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            if m.msuccess:
                t["nextIndex"] = fset2(s["nextIndex"], i, j, max(m.mmatchIndex, 1))
                t["matchIndex"] = fset2(s["matchIndex"], i, j, m.mmatchIndex)
            else:
                t["nextIndex"] = fset2(s["nextIndex"], i, j, max(s["nextIndex"][i][j] - 2, 1))
            t["pendingResponse"] = fset2(s["pendingResponse"], i, j, False)
            t["messages"] = msgs
            yield t

    ref_hrvresp = ("m", lambda sp, s: sp.HandleRequestVoteResponse(s))
    ref_haeresp = ("m", lambda sp, s: sp.HandleAppendEntriesResponse(s))
    ref_rejae = ("m", lambda sp, s: sp.RejectAppendEntriesRequest(s))
    return {
        "raft_hrvresp_text_n3v1e1": {"HRVRespText": ref_hrvresp},
        "raft_hrvresp_all_n2v1e2": {"HRVRespAll": ("m", hrvresp_all)},
        "raft_hrvreq_nolog_n2v1e2": {"HRVReqNoLog": ("m", hrvreq_nolog)},
        "raft_rejae_text_n2v2e2": {"RejAEText": ref_rejae},
        "raft_rejae_lenidx_n2v2e2": {"RejAELen": ("m", rejae_lenidx)},
        "raft_updateterm_stay_n2v1e2": {"UpdateTermStay": ("m", updateterm_stay)},
        "raft_two_handlers_n2v1e2r1": {"HRVRespAll": ("m", hrvresp_all), "RejAEText": ref_rejae},
        "flex_hrvresp_all_n2v1e2": {"HRVRespAll": ("m", hrvresp_all)},
        "fsync_rejae_text_n2v1e2r1": {"RejAEText": ref_rejae},
        "fsync_hrvreq_nolog_n2v1e2r1": {"HRVReqNoLog": ("m", hrvreq_nolog)},
        "raft_haeresp_text_n3v1e1": {"HAERespText": ref_haeresp},
        "raft_haeresp_resend_n2v2e2": {"HAERespResend": ("m", haeresp_resend)},
        "fsync_haeresp_text_n2v1e2r1": {"HAERespText": ref_haeresp},
    }


def handlers():
    """--handlers: Next with message handlers the front end compiles whole
    (cfgs.HANDLERS), by the Python oracle with the same handlers written in
    Python (_handler_py); the handlers written out from the reference text are
    also checked against the oracle's own (built-in) space.  Pinned by the
    Python oracle alone (the C oracle has no configurable actions)."""
    py = _handler_py()
    path = os.path.join(HERE, "handlers.json")
    only = [a.split("=", 1)[1].split(",") for a in sys.argv if a.startswith("--only=")]
    out = json.load(open(path)) if only and os.path.exists(path) else {}
    for name, module, kw, nxt, acts, md in HANDLERS:
        if only and name not in only[0]:
            continue
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        p = bfs(make_spec(module, cfg, next_order=nxt, defined=py[name]), max_depth=md or None)
        out[name] = dict(module=module, cfg=txt, next=list(nxt), actions=[list(a) for a in acts], max_depth=md,
                         generated=p.generated, distinct=p.distinct, depth=p.depth, status=p.status,
                         violated=getattr(p, "violated", None), levels=[list(x) for x in p.levels],
                         hidden_same_level=p.hidden_same_level, max_msgs=p.max_msgs,
                         trace_len=len(p.trace) if getattr(p, "trace", None) else None, pinned_by="pyoracle")
        print(name, p.generated, p.distinct, p.depth, p.status, getattr(p, "violated", None), p.hidden_same_level,
              "%.1fs" % p.seconds, flush=True)
    out = {k: v for k, v in out.items() if k in {e[0] for e in HANDLERS}}
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def main():
    if "--handlers" in sys.argv:
        return handlers()
    if "--effects" in sys.argv:
        return effects()
    if "--guards" in sys.argv:
        return guards()
    if "--frontend" in sys.argv:
        return frontend()
    if "--extras" in sys.argv:
        return extras()
    if "--ladders" in sys.argv or "--ladder-one" in sys.argv:
        return ladders()
    if "--flex-restart" in sys.argv:
        return flex_restart()
    if "--variant2" in sys.argv:
        return variant2()
    if "--order" in sys.argv:
        return order()
    if "--shipped-one" in sys.argv:
        return shipped()
    if "--unsafe" in sys.argv:
        return unsafe()
    if "--n5" in sys.argv or "--n5-unsafe" in sys.argv:
        return n5()
    out = {}
    for name, module, kw in SMALL:
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=4)
        spec = make_spec(module, cfg)
        p = bfs(spec)
        pr = (p.generated, p.distinct, p.depth, p.status, [list(x) for x in p.levels])
        cr = (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"])
        if pr != cr:
            raise SystemExit("oracles disagree on %s: py=%s c=%s" % (name, pr[:4], cr[:4]))
        out[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"],
                         depth=c["depth"], status=c["status"], levels=c["levels"],
                         action_counts=c["action_counts"], max_msgs=c["max_msgs"],
                         hidden_same_level=c["hidden_same_level"], pinned_by="pyoracle==coracle")
        print(name, c["generated"], c["distinct"], c["depth"], flush=True)
    with open(os.path.join(HERE, "small.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    med = {}
    for name, module, kw in MEDIUM:
        txt = cfg_text(module, **kw)
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=8, extra=["--trace"])
        med[name] = dict(module=module, cfg=txt, generated=c["generated"], distinct=c["distinct"],
                         depth=c["depth"], status=c["status"], levels=c["levels"], violated=c["violated"],
                         action_counts=c["action_counts"], max_msgs=c["max_msgs"],
                         hidden_same_level=c["hidden_same_level"], pinned_by="coracle",
                         trace_len=len(c.get("trace", [])))
        print(name, c["generated"], c["distinct"], c["depth"], c["status"], c["violated"], flush=True)
    with open(os.path.join(HERE, "medium.json"), "w") as f:
        json.dump(med, f, indent=1, sort_keys=True)
    if "--shipped" in sys.argv:
        shipped()


def shipped():
    """--shipped: every shipped cfg; --shipped-one NAME: one, merged into shipped.json."""
    only = sys.argv[sys.argv.index("--shipped-one") + 1] if "--shipped-one" in sys.argv else None
    sp = os.path.join(HERE, "shipped.json")
    ship = json.load(open(sp)) if (only and os.path.exists(sp)) else {}
    for name, module, path in SHIPPED:
        if only and name != only:
            continue
        with open(os.path.join(ROOT, path)) as fh:
            txt = fh.read()
        cfg = parse_cfg(txt)
        c = run_c.run(module, cfg["constants"], cfg["invariants"], threads=8)
        ship[name] = dict(module=module, cfg_path=path, generated=c["generated"], distinct=c["distinct"],
                          depth=c["depth"], status=c["status"], levels=c["levels"],
                          action_counts=c["action_counts"], max_msgs=c["max_msgs"],
                          hidden_same_level=c["hidden_same_level"],
                          hidden_cross_level=c["hidden_cross_level"], pinned_by="coracle",
                          oracle_seconds=c["seconds"])
        print(name, c["generated"], c["distinct"], c["depth"], flush=True)
    with open(os.path.join(HERE, "shipped.json"), "w") as f:
        json.dump(ship, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
