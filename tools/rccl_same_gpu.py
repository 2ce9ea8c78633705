"""Probe: two RCCL ranks of rmc_check_sharded on ONE GPU (device 0), launched
with torch.distributed.run.  Exercises the RCCL transport's multi-rank path
on a 1-GPU box if RCCL permits two ranks per device."""
import json
import os
import sys

import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-tlaplus_amd"))
import raftmc  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
g = json.load(open(os.path.join(ROOT, "tests", "golden", "small.json")))["raft_n3v1e1"]
uid = [raftmc.comm_unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)
m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
r = m.check_sharded(rank, world, 0, uid[0], chunk_parents=100)
ok = (r["generated"], r["distinct"], r["depth"], r["levels"]) == (g["generated"], g["distinct"], g["depth"], g["levels"])
print("rank", rank, "ok" if ok else "MISMATCH", r["generated"], r["distinct"], r["depth"], flush=True)
dist.destroy_process_group()
sys.exit(0 if ok else 1)
