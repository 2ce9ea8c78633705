#!/usr/bin/env python3
"""Normalised-text fingerprints of the reference specs the checker lowers by
hand (rmc_engine.cpp `known_spec_hash`): block and line comments removed, all
whitespace removed, FNV-1a 64.  Run in the build container, where the
reference is mounted, to regenerate the table:
    python tools/spec_hashes.py /root/reference/specifications
"""
import os
import sys

SPECS = {"Raft": "standard-raft/Raft.tla", "FlexibleRaft": "flexible-raft/FlexibleRaft.tla",
         "PullRaft": "pull-raft/PullRaft.tla", "RaftFsync": "raft-and-fsync/RaftFsync.tla",
         "PullRaftVariant2": "pull-raft/PullRaftVariant2.tla", "KRaft": "pull-raft/KRaft.tla"}


def normalise(t):
    out, depth, i = [], 0, 0
    while i < len(t):
        if t.startswith("(*", i):
            depth += 1
            i += 2
        elif depth and t.startswith("*)", i):
            depth -= 1
            i += 2
        elif depth:
            i += 1
        elif t.startswith("\\*", i):
            while i < len(t) and t[i] != "\n":
                i += 1
        else:
            if not t[i].isspace():
                out.append(t[i])
            i += 1
    return "".join(out)


def fnv1a64(s):
    h = 0xcbf29ce484222325
    for b in s.encode():
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/specifications"
    for mod, rel in SPECS.items():
        print('{"%s", 0x%016xULL},' % (mod, fnv1a64(normalise(open(os.path.join(root, rel)).read()))))
