"""Run the C oracle (oracle/_build/rmc_oracle) on a TLC cfg.  TEST INFRASTRUCTURE ONLY."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "_build", "rmc_oracle")


def cfg_args(module, consts, invariants=None):
    a = ["--spec", module, "--servers", str(len(consts["Server"])),
         "--values", str(len(consts["Value"])),
         "--max-elections", str(int(consts["MaxElections"])),
         "--max-restarts", str(int(consts["MaxRestarts"]))]
    if module == "FlexibleRaft":
        a += ["--eq", str(int(consts["ElectionQuorumSize"])),
              "--rq", str(int(consts["ReplicationQuorumSize"]))]
    if module == "RaftFsync":
        a += ["--lfae", str(int(bool(consts["LeaderFsyncBeforeAppendEntries"]))),
              "--lfiq", str(int(bool(consts["LeaderFsyncBeforeIncludeInQuorum"]))),
              "--ffbr", str(int(bool(consts["FollowerFsyncBeforeReply"])))]
    if invariants:
        a += ["--inv", ",".join(invariants)]
    return a


def run(module, consts, invariants=None, threads=1, extra=(), timeout=None):
    cmd = [BIN] + cfg_args(module, consts, invariants) + ["--threads", str(threads)] + list(extra)
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout).stdout
    return json.loads(out)


KRAFT_BIN = os.path.join(HERE, "_build", "kraft_oracle")


def run_kraft(consts, invariants=None, max_states=0, timeout=None):
    """The C++ KRaft oracle (oracle/cengine/kraft_oracle.cpp) on a KRaft cfg's constants."""
    cmd = [KRAFT_BIN, "--servers", str(len(consts["Server"])), "--values", str(len(consts["Value"])),
           "--max-elections", str(int(consts["MaxElections"])), "--max-restarts", str(int(consts["MaxRestarts"]))]
    if invariants:
        cmd += ["--inv", ",".join(invariants)]
    if max_states:
        cmd += ["--max-states", str(int(max_states))]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout).stdout
    return json.loads(out)
