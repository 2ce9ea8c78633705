"""The fingerprint-set insert microbenchmark runs and reaches
the loads it reports: raft-tlaplus_amd/build/fpset_bench, small table."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "raft-tlaplus_amd", "build", "fpset_bench")


def test_fpset_bench_binary_built():
    assert os.access(BIN, os.X_OK), "build fpset_bench first (make -C raft-tlaplus_amd)"


@pytest.mark.gpu
def test_fpset_bench_small():
    out = subprocess.run([BIN, "-slots_log2", "20", "-batch", "65536", "-loads", "0.25,0.5,0.75"],
                         capture_output=True, text=True, timeout=60, check=True).stdout
    rows = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert [round(r["load"], 2) for r in rows] == [0.25, 0.5, 0.75]
    for r in rows:
        assert r["table_full"] == 0
        assert abs(r["new"] / r["batch"] - (1 - r["dup"])) < 0.02  # duplicate ratio as asked
        assert r["inserts_per_s"] > 0
