"""The packed message layout (raft-tlaplus_amd/csrc/rmc_spec.h): codec round
trip, field positions, and that unsigned order of packed words IS TLC's
record order (so a sorted word array is TLC's DOMAIN enumeration order).
Runs the library's host code only; no GPU."""
import itertools
import random

import pytest

import raftmc
from oracle.pyoracle.tlc import NIL, Rec, tlc_key

RV, RVR, AE, AER, LN, PE, PER = range(7)
NAMES = {RV: "RequestVoteRequest", RVR: "RequestVoteResponse", AE: "AppendEntriesRequest",
         AER: "AppendEntriesResponse", LN: "LeaderNotifyRequest", PE: "PullEntriesRequest",
         PER: "PullEntriesResponse"}


def random_msg(rng, spec_pull, variant2=False):
    t = rng.choice([RV, RVR, LN, PE, PER] if spec_pull else [RV, RVR, AE, AER])
    f = dict(type=t, term=rng.randint(0, 7), src=rng.randint(0, 4), dst=rng.randint(0, 4), count=rng.randint(0, 7))
    if t in (RV, PE):
        f.update(lli=rng.randint(0, 5), llt=rng.randint(0, 7))
    elif t == RVR:
        f.update(granted=rng.randint(0, 1))
        if variant2:
            f.update(lli=rng.randint(0, 5), llt=rng.randint(0, 7))
    elif t == LN and variant2:
        if rng.randint(0, 2) == 0:
            f.update(lcenil=1)
        else:
            f.update(lci=rng.randint(0, 5), lct=rng.randint(0, 7))
    elif t == AE:
        f.update(pli=rng.randint(0, 5), plt=rng.randint(0, 7), nent=rng.randint(0, 1), commit=rng.randint(0, 5))
        if f["nent"]:
            f.update(eterm=rng.randint(1, 7), evalue=rng.randint(0, 3))
    elif t == AER:
        f.update(success=rng.randint(0, 1), midx=rng.randint(0, 5))
    elif t == PER:
        f.update(success=rng.randint(0, 1))
        if f["success"]:
            f.update(nent=1, eterm=rng.randint(1, 7), evalue=rng.randint(0, 3), commit=rng.randint(0, 5))
        else:
            f.update(lci=rng.randint(0, 5), lct=rng.randint(0, 7))
    return f


def as_record(f, variant2=False):
    """The TLA+ record value (oracle representation) for the field dict."""
    t = f["type"]
    base = dict(mtype=NAMES[t], mterm=f["term"], msource=f["src"], mdest=f["dst"])
    ent = (Rec(term=f.get("eterm", 0), value=f.get("evalue", 0)),) if f.get("nent") else ()
    if t in (RV, PE):
        base.update(mlastLogIndex=f["lli"], mlastLogTerm=f["llt"])
    elif t == RVR:
        base.update(mvoteGranted=bool(f["granted"]))
        if variant2:  # PullRaftVariant2.tla:317-323
            base.update(mlastLogIndex=f["lli"], mlastLogTerm=f["llt"])
    elif t == LN and variant2:  # PullRaftVariant2.tla:369-377: Nil or [index, term]
        base.update(mlastCommonEntry=NIL if f.get("lcenil") else Rec(index=f["lci"], term=f["lct"]))
    elif t == AE:
        base.update(mprevLogIndex=f["pli"], mprevLogTerm=f["plt"], mentries=ent, mcommitIndex=f["commit"])
    elif t == AER:
        base.update(msuccess=bool(f["success"]), mmatchIndex=f["midx"])
    elif t == PER:
        base.update(msuccess=bool(f["success"]))
        if f["success"]:
            base.update(mentries=ent, mcommitIndex=f["commit"])
        else:
            base.update(mlastCommonEntry=Rec(index=f["lci"], term=f["lct"]))
    return Rec(**base)


@pytest.mark.parametrize("pull", [False, True])
def test_codec_roundtrip_and_positions(pull):
    rng = random.Random(7 + pull)
    for _ in range(3000):
        f = random_msg(rng, pull)
        _, ok = raftmc.encode_msg(3 if pull else 0, **f)
        assert ok, f


@pytest.mark.parametrize("pull", [False, True])
def test_packed_order_is_tlc_order(pull):
    rng = random.Random(11 + pull)
    msgs = [random_msg(rng, pull) for _ in range(400)]
    for a, b in itertools.combinations(msgs, 2):
        wa, _ = raftmc.encode_msg(3 if pull else 0, **a)
        wb, _ = raftmc.encode_msg(3 if pull else 0, **b)
        ka, kb = tlc_key(as_record(a)), tlc_key(as_record(b))
        if ka == kb:
            assert wa >> 3 == wb >> 3
        else:
            assert (wa >> 3 < wb >> 3) == (ka < kb), (a, b)


def test_variant2_codec_roundtrip_and_positions():
    rng = random.Random(23)
    for _ in range(3000):
        f = random_msg(rng, True, variant2=True)
        _, ok = raftmc.encode_msg(4, **f)
        assert ok, f


def test_variant2_packed_order_is_tlc_order():
    """PullRaftVariant2's records: RVResp grows to 7 fields, LeaderNotify's
    mlastCommonEntry is Nil (below every record) or a record."""
    rng = random.Random(29)
    msgs = [random_msg(rng, True, variant2=True) for _ in range(400)]
    for a, b in itertools.combinations(msgs, 2):
        wa, _ = raftmc.encode_msg(4, **a)
        wb, _ = raftmc.encode_msg(4, **b)
        ka, kb = tlc_key(as_record(a, True)), tlc_key(as_record(b, True))
        if ka == kb:
            assert wa >> 3 == wb >> 3
        else:
            assert (wa >> 3 < wb >> 3) == (ka < kb), (a, b)
