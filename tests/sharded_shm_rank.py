"""One rank of a multi-process fingerprint-sharded check over the shared-memory
transport (rmc_check_sharded_shm); launched by tests/test_gpu_sharded_mp.py.
argv: rank world shm_name fixture_file fixture_name chunk [host_frontier] -> prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "raft-tlaplus_amd"))
import raftmc  # noqa: E402

rank, world, name, fx, key, chunk = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5], sys.argv[6]
extra = {"host_frontier": int(sys.argv[7])} if len(sys.argv) > 7 else {}
g = json.load(open(os.path.join(HERE, "golden", fx)))[key]
if "cfg" in g:
    m = raftmc.Model(module=g["module"], cfg_text=g["cfg"])
else:  # shipped.json: the restated reference cfg under configs/
    root = os.path.dirname(HERE)
    m = raftmc.Model(module=g["module"], cfg_path=os.path.join(root, g["cfg_path"]))
try:
    r = m.check_sharded_shm(int(rank), int(world), 0, name, chunk_parents=int(chunk), **extra)
except raftmc.RaftmcError as e:
    print(json.dumps(dict(rank=int(rank), error=str(e))), flush=True)
    sys.exit(3)
r.pop("trace", None)
print(json.dumps(dict(rank=int(rank), **{k: r[k] for k in ("generated", "distinct", "depth", "status", "violated",
                                                             "levels", "hidden_var_collisions", "message")})),
      flush=True)
