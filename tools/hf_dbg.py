"""Debug: the tail of tests/test_gpu_configs.py in suite order, printing
device free memory (hipMemGetInfo via torch) after every check and release."""
import os, sys, time
sys.path.insert(0, 'raft-tlaplus_amd')
import torch
import raftmc

F = ('RaftFsync', 'configs/RaftFsync_n3v1e2r1.cfg')
R = ('Raft', 'configs/Raft_n3v2e2.cfg')


def free(tag):
    f, t = torch.cuda.mem_get_info()
    print('%-28s free %.1f / %.1f GiB' % (tag, f / 2**30, t / 2**30), flush=True)


def run(tag, spec, fn):
    t0 = time.time()
    r = fn(raftmc.Model(module=spec[0], cfg_path=spec[1]))
    print(tag, r['generated'], r['distinct'], r['depth'], r['status'], r['message'], r.get('device_bytes'),
          '%.1fs' % (time.time() - t0), flush=True)
    free('after ' + tag)


free('start')
run('full R', R, lambda m: m.check())
raftmc.release_device_memory(); free('release')
run('fp128 R', R, lambda m: m.check(fp_bits=128))
run('logical2 F', F, lambda m: m.check_logical(2))
run('logical2 R', R, lambda m: m.check_logical(2))
raftmc.release_device_memory(); free('release')
run('hf F', F, lambda m: m.check(host_frontier=1))
raftmc.release_device_memory(); free('release')
time.sleep(5); free('release+5s')
os.environ['RMC_VERBOSE'] = '1'
run('hf R', R, lambda m: m.check(host_frontier=1))
