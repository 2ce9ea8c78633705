"""Debug: tests/test_gpu_configs.py's checks in its order, printing the
device's free HBM (hipMemGetInfo) and rmc_result.device_bytes after every
check and every release_device_memory()."""
import ctypes, json, os, sys, time
sys.path.insert(0, 'raft-tlaplus_amd')
import raftmc

LAD = json.load(open('tests/golden/ladders.json'))
EXH = json.load(open('tests/golden/exhausted.json'))
BEYOND = ["raft_n3v2e3_cfg2", "fsync_n3v2e3r1_cfg5"]
hip = ctypes.CDLL("libamdhip64.so")


def free():
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
    return f.value / 2**30


def model(g):
    return raftmc.Model(module=g["module"], cfg_path=g["cfg_path"])


def run(tag, fn):
    t0 = time.time()
    r = fn()
    print('%-34s %-9s depth %2d dev %6.1f GiB  free %6.1f GiB  %.1fs %s' % (
        tag, r['status'], r['depth'], r.get('device_bytes', 0) / 2**30, free(), time.time() - t0,
        r.get('message', '')[:90]), flush=True)


def release(tag):
    raftmc.release_device_memory()
    print('%-34s release                                   free %6.1f GiB' % (tag, free()), flush=True)


print('start free %.1f' % free(), flush=True)
if os.environ.get('DBG_SHARDS'):  # the per-shard breakdown of the bench rung at W = 1 (single), 2, 4
    os.environ['RMC_VERBOSE'] = '1'
    g = EXH["raft_n3v2e2_bench"]
    run('single', lambda: model(g).check())
    for W in (2, 4):
        run('logical %d' % W, lambda: model(g).check_logical(W, verbose=True))
    del os.environ['RMC_VERBOSE']
    release('after shards')
    if os.environ['DBG_SHARDS'] == 'only':
        sys.exit(0)
for n in sorted(LAD):
    run('prefix ' + n, lambda: model(LAD[n]).check(max_depth=LAD[n]["depth"]))
for n in BEYOND:
    run('prefix logical ' + n, lambda: model(LAD[n]).check_logical(2, max_depth=LAD[n]["depth"]))
for n in BEYOND:
    run('prefix hf ' + n, lambda: model(LAD[n]).check(max_depth=LAD[n]["depth"], host_frontier=1))
for n in sorted(EXH):
    run('full ' + n, lambda: model(EXH[n]).check())
for n in sorted(EXH):
    release('fp128 ' + n)
    run('fp128 ' + n, lambda: model(EXH[n]).check(fp_bits=128))
for n in sorted(EXH):
    run('logical2 ' + n, lambda: model(EXH[n]).check_logical(2))
for n in sorted(EXH):
    release('hf ' + n)
    run('hf ' + n, lambda: model(EXH[n]).check(host_frontier=1))
