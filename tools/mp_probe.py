import json, os, subprocess, sys, uuid
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
cases = [(2, "small.json", "raft_n3v1e1", 97), (3, "small.json", "raft_n3v1e1", 0), (2, "small.json", "pull_n3v2e1", 0),
         (2, "small.json", "pull_n3v2e1", 97), (3, "small.json", "pull_n3v2e1", 0), (2, "small.json", "raft_n2v2e2", 7)]
for world, fx, key, chunk in cases:
    g = json.load(open(os.path.join(ROOT, "tests", "golden", fx)))[key]
    name = "rmc_probe_" + uuid.uuid4().hex[:10]
    ps = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "sharded_shm_rank.py"), str(r), str(world), name, fx, key, str(chunk)],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    res = []
    for p in ps:
        o, e = p.communicate(timeout=200)
        res.append(o.strip().splitlines()[-1] if o.strip() else "NO OUTPUT " + e[-300:])
    want = (g["generated"], g["distinct"], g["depth"], g["status"])
    print(world, key, chunk, "want", want, flush=True)
    for line in res:
        print("   ", line[:300], flush=True)
