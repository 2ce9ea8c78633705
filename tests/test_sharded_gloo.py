"""The multi-GPU (fingerprint-sharded) protocol, world_size 2 over gloo on CPU.

tests/sharded_protocol.py restates rmc_sharded.cpp's level protocol
(block-cyclic TLC-order layout, owner dedupe with first-in-TLC-order wins,
reverse win flags, redistribution by global position) over real
torch.distributed collectives; its counts must equal the single-process
oracle fixtures bit for bit.  The GPU implementation of the same protocol is
tested against the same fixtures in tests/test_gpu_sharded.py.
"""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = json.load(open(os.path.join(HERE, "golden", "small.json")))
CASES = [("pull_n3v1e1", 3), ("raft_n2v1e2", 16), ("fsync_n2v1e2r1", 64), ("flex_n2v1e2", 5)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    import torch.distributed as dist
    from oracle.pyoracle import make_spec
    from oracle.pyoracle.cfg import parse_cfg
    from sharded_protocol import sharded_bfs
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    res = {}
    for name, ch in CASES:
        g = SMALL[name]
        res[name] = sharded_bfs(make_spec(g["module"], parse_cfg(g["cfg"])), ch)
    dist.destroy_process_group()
    with open(os.path.join(outdir, "rank%d.json" % rank), "w") as f:
        json.dump(res, f)


@pytest.mark.timeout(600)
def test_sharded_protocol_world2_matches_oracle(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for rank in range(world):
        got = json.load(open(tmp_path / ("rank%d.json" % rank)))
        for name, _ in CASES:
            g, r = SMALL[name], got[name]
            assert (r["generated"], r["distinct"], r["depth"], r["status"]) == \
                (g["generated"], g["distinct"], g["depth"], g["status"]), (rank, name)
            assert r["levels"] == g["levels"], (rank, name)
