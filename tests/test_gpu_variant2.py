"""GPU: PullRaftVariant2 through the C ABI against the
oracle fixtures (tests/golden/variant2.json, shipped.json): every per-level
count and the hidden-variable collision count, over chunk sizes, 128-bit
fingerprints and the fingerprint-sharded protocol."""
import json
import os

import pytest

import raftmc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
V2 = json.load(open(os.path.join(HERE, "golden", "variant2.json")))
SHIPPED = json.load(open(os.path.join(HERE, "golden", "shipped.json")))

pytestmark = pytest.mark.gpu


def same(r, g):
    assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
        (g["generated"], g["distinct"], g["depth"], g["status"])
    assert r["levels"] == g["levels"]
    assert r["hidden_var_collisions"] == g["hidden_same_level"]


@pytest.mark.parametrize("name", sorted(V2))
@pytest.mark.parametrize("chunk", [0, 7, 1000])
def test_variant2_matches_oracle(name, chunk):
    g = V2[name]
    same(raftmc.check_text(g["module"], g["cfg"], chunk_parents=chunk), g)


@pytest.mark.parametrize("name", ["pull2_n3v1e2", "pull2_n5v1e1"])
def test_variant2_fp128(name):
    g = V2[name]
    same(raftmc.check_text(g["module"], g["cfg"], fp_bits=128), g)


@pytest.mark.parametrize("name", ["pull2_n3v2e1", "pull2_n3v1e2r1"])
@pytest.mark.parametrize("shards,chunk", [(2, 0), (3, 55)])
def test_variant2_logical_shards(name, shards, chunk):
    g = V2[name]
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
    same(m.check_logical(shards, chunk_parents=chunk), g)


def test_variant2_shipped_cfg():
    """PullRaftVariant2.cfg's constants: 891 same-level hidden-variable collisions
    in TLC order (2,615 if the last successor won)."""
    g = SHIPPED["PullRaftVariant2_cfg"]
    m = raftmc.Model(module="PullRaftVariant2", cfg_path=os.path.join(ROOT, g["cfg_path"]))
    for kw in (dict(), dict(chunk_parents=10000)):
        r = m.check(**kw)
        assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == \
            (g["generated"], g["distinct"], g["depth"], g["levels"])
        assert r["hidden_var_collisions"] == g["hidden_same_level"] == 891
