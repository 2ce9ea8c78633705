import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "raft-tlaplus_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running (full shipped configs)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


# RMC_TEST_MEMLOG=<file>: append the device's free HBM after every test
# (hipMemGetInfo through the HIP runtime directly) -- for finding a test that
# leaves device memory behind.
if os.environ.get("RMC_TEST_MEMLOG"):
    import ctypes
    import time

    @pytest.fixture(autouse=True)
    def _memlog(request):
        yield
        try:
            hip = ctypes.CDLL("libamdhip64.so")
            f, t = ctypes.c_size_t(), ctypes.c_size_t()
            series = []
            # RMC_TEST_MEMLOG_POLL=<s>: also poll once a second for that long
            for k in range(1 + int(os.environ.get("RMC_TEST_MEMLOG_POLL", "0"))):
                if k:
                    time.sleep(1)
                hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
                series.append("%.1f" % (f.value / 2**30))
            with open(os.environ["RMC_TEST_MEMLOG"], "a") as out:
                out.write("%-90s free GiB %s\n" % (request.node.nodeid, " ".join(series)))
        except OSError:
            pass
