"""KRaft (pull-raft/KRaft.tla) on the CPU: the Python
oracle on the committed fixtures (tests/golden/kraft.json, made by
tests/golden/make_kraft.py), the lowered actions replayed on the host
(rmc_spec.h kr_*, the code the kernels run), the CPU engine (same layout and
first-in-TLC-order rule as the GPU path) and the packed record order.

Parity: pinned by two independent restatements, the Python oracle and the
C++ oracle (oracle/cengine/kraft_oracle.cpp); the lowering is a third."""
import json
import os

import pytest

import raftmc
from oracle.pyoracle import make_spec
from oracle.pyoracle.cfg import parse_cfg
from oracle.pyoracle.tlc import bfs

HERE = os.path.dirname(os.path.abspath(__file__))
KR = json.load(open(os.path.join(HERE, "golden", "kraft.json")))
FULL = sorted(k for k in KR if KR[k]["status"] != "truncated" and not KR[k].get("slow"))
FAST = sorted(k for k in FULL if KR[k]["distinct"] <= 5000)


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    if g["status"] == "ok":
        assert r["levels"] == g["levels"]
        assert r["hidden_var_collisions"] == g["hidden_same_level"]
    else:
        assert r["violated"] == g["violated"]


@pytest.mark.parametrize("name", FAST)
def test_python_oracle_reproduces_fixture(name):
    g = KR[name]
    p = bfs(make_spec("KRaft", parse_cfg(g["cfg"])))
    assert (p.generated, p.distinct, p.depth, p.status) == (g["generated"], g["distinct"], g["depth"], g["status"])
    if g["status"] == "ok":
        assert [list(x) for x in p.levels] == g["levels"]


@pytest.mark.parametrize("name", FULL)
def test_host_replay_of_lowered_actions(name):
    g = KR[name]
    r = raftmc.Model(module="KRaft", cfg_text=g["cfg"]).selftest_host_bfs()
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    if g["status"] == "ok":
        assert r["levels"] == g["levels"]


def test_host_replay_shipped_cfg_prefix():
    """KRaft.cfg's constants (N=3, V=1, MaxElections=2): the oracle's first levels."""
    g = KR["KRaft_cfg_prefix"]
    r = raftmc.Model(module="KRaft", cfg_text=g["cfg"]).selftest_host_bfs(max_distinct=g["distinct"])
    n = len(g["levels"])
    assert r["levels"][:n] == g["levels"]


@pytest.mark.parametrize("name", FULL)
@pytest.mark.parametrize("workers,chunk", [(8, 0), (3, 97)])
def test_cpu_engine(name, workers, chunk):
    g = KR[name]
    same(raftmc.Model(module="KRaft", cfg_text=g["cfg"]).check_cpu(workers=workers, chunk_parents=chunk), g)


def test_fixtures_exercise_the_kraft_actions():
    """Every KRaft action fires in the fixtures, and the unsafe ones reach IllegalState."""
    seen = {}
    for g in KR.values():
        for k, v in g["action_counts"].items():
            seen[k] = seen.get(k, 0) + v
    for a in ("RequestVote", "HandleRequestVoteRequest", "HandleRequestVoteResponse", "BecomeLeader",
              "ClientRequest", "RejectFetchRequest", "DivergingFetchRequest", "AcceptFetchRequest",
              "HandleBeginQuorumRequest", "SendFetchRequest", "HandleSuccessFetchResponse",
              "HandleDivergingFetchResponse", "HandleErrorFetchResponse", "Restart"):
        assert seen.get(a, 0) > 0, a
    assert any(g.get("violated") == "NoIllegalState" for g in KR.values())


def test_kraft_bounds_are_checked():
    """Records pack into one DOMAIN word only for 2-bit epochs and offsets."""
    from cfgs import kraft_cfg_text
    with pytest.raises(Exception):
        raftmc.Model(module="KRaft", cfg_text=kraft_cfg_text(n=3, v=1, E=3))


def _random_kraft_record(rng, N=3, V=3):
    """A random KRaft message: the oracle's Rec (oracle/pyoracle/kraft.py) and the probe's fields."""
    from oracle.pyoracle import kraft as K
    from oracle.pyoracle.tlc import Rec
    errs = [K.FENCED, K.NILE, K.NOTLEADER, K.UNKNOWNLEADER]
    cls = rng.randrange(7)
    src, dst = rng.sample(range(N), 2)
    ep = rng.randrange(4)
    f = dict(cls=cls, src=src, dst=dst, epoch=ep, count=1)
    if cls == 0:
        return Rec(mtype=K.BQREQ, mepoch=ep, msource=src, mdest=dst), f
    if cls == 1:
        e = rng.randrange(4)
        f["err"] = e
        return Rec(mtype=K.BQRESP, mepoch=ep, merror=errs[e], msource=src, mdest=dst), f
    if cls == 2:
        a, b = rng.randrange(4), rng.randrange(4)
        f.update(f1=a, f2=b)
        if rng.randrange(2):
            f["granted"] = 1
            return Rec(mtype=K.RVREQ, mepoch=ep, mlastLogEpoch=a, mlastLogOffset=b, msource=src, mdest=dst), f
        return Rec(mtype=K.FREQ, mepoch=ep, mfetchOffset=a, mlastFetchedEpoch=b, msource=src, mdest=dst), f
    ld = rng.randrange(-1, N)
    f["leader"] = ld
    if cls == 3:
        e, gr = rng.randrange(4), rng.randrange(2)
        f.update(err=e, granted=gr)
        return Rec(mtype=K.RVRESP, mepoch=ep, mleader=ld, mvoteGranted=bool(gr), merror=errs[e],
                   msource=src, mdest=dst), f
    ce, cfo, clfe, hwm = rng.randrange(4), rng.randrange(4), rng.randrange(4), rng.randrange(4)
    f.update(cepoch=ce, cfo=cfo, clfe=clfe, hwm=hwm)
    corr = Rec(mtype=K.FREQ, mepoch=ce, mfetchOffset=cfo, mlastFetchedEpoch=clfe, msource=dst, mdest=src)
    common = dict(mtype=K.FRESP, mepoch=ep, mleader=ld, mhwm=hwm, msource=src, mdest=dst, correlation=corr)
    if cls == 4:
        e = rng.choice([0, 2, 3])
        f["err"] = e
        return Rec(mresult=K.NOTOK, merror=errs[e], **common), f
    if cls == 5:
        n = rng.randrange(2)
        ee, ev = (rng.randrange(4), rng.randrange(V)) if n else (0, 0)
        f.update(elen=n, eepoch=ee, evalue=ev)
        ents = (Rec(epoch=ee, value=ev),) if n else ()
        return Rec(mresult=K.OK, merror=K.NILE, mentries=ents, **common), f
    de, dd = rng.randrange(4), rng.randrange(4)
    f.update(divend=de, divepoch=dd)
    return Rec(mresult=K.DIVERGING, merror=K.NILE, mdivergingEpoch=dd, mdivergingEndOffset=de, **common), f


def test_kraft_packed_order_is_tlc_order():
    """Packed words sort exactly as TLC orders the records (field count, then
    sorted field names with values; model values by name; Nil below servers),
    so a row's sorted DOMAIN is TLC's enumeration order; and the codec reads
    every field back."""
    import random
    from oracle.pyoracle.tlc import tlc_key
    rng = random.Random(7)
    recs = {}
    for _ in range(4000):
        r, f = _random_kraft_record(rng)
        w, ok = raftmc.encode_kmsg(**f)
        assert ok, f
        if r in recs:
            assert recs[r] == w >> 3
        recs[r] = w >> 3
    by_tlc = sorted(recs, key=tlc_key)
    words = [recs[r] for r in by_tlc]
    assert words == sorted(words) and len(set(words)) == len(words)


@pytest.mark.parametrize("name", sorted(k for k in KR if not KR[k].get("slow")))
def test_c_oracle_reproduces_fixture(name):
    """The independent C++ restatement (oracle/cengine/kraft_oracle.cpp) agrees."""
    from oracle import run_c
    g = KR[name]
    cfg = parse_cfg(g["cfg"])
    c = run_c.run_kraft(cfg["constants"], cfg["invariants"], max_states=g.get("max_states", 0))
    assert (c["generated"], c["distinct"], c["depth"], c["status"], c["levels"], c["hidden_same_level"],
            c["action_counts"]) == (g["generated"], g["distinct"], g["depth"], g["status"], g["levels"],
                                    g["hidden_same_level"], g["action_counts"])


def test_kraft_hand_derived_first_levels():
    """Known answers derived by hand from KRaft.tla for KRaft.cfg's constants
    (N=3, V={v1}, MaxElections=2), independent of every restatement:
    level 1 = Init (:397-415), 1 state.
    level 2: only RequestVote(i) is enabled (all Unattached, :441; no messages,
      no leader): 3 successors, one orbit under symmServers -> [3, 1].
    level 3, from n1 Candidate at epoch 2 with RVReqs to n2, n3: RequestVote(n1)
      again (Candidate, electionCtr 1 < 2), RequestVote(n2), RequestVote(n3),
      HandleRequestVoteRequest on each RVReq (epoch 2 > 1: Unattached -> Voted,
      grant) -> 5 successors; n2/n3 are symmetric, so 3 distinct -> [5, 3]."""
    g = KR["KRaft_cfg_prefix"]
    assert g["levels"][:3] == [[1, 1], [3, 1], [5, 3]]
    r = raftmc.Model(module="KRaft", cfg_text=g["cfg"]).selftest_host_bfs(max_distinct=5)
    assert r["levels"][:3] == [[1, 1], [3, 1], [5, 3]]
