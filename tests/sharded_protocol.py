"""The fingerprint-sharded BFS protocol of raft-tlaplus_amd/csrc/rmc_sharded.cpp,
restated over torch.distributed (gloo) for CPU tests.  TEST INFRASTRUCTURE.

Same decisions as the GPU driver, so a world_size > 1 run must reproduce the
single-process oracle's counts exactly:
  * a level's states are laid out block-cyclically by global TLC position g:
    shard (g // CH) % W, local index (g // (W*CH))*CH + g % CH;
  * round c expands every shard's c-th local block (one contiguous global
    range, increasing with c);
  * a candidate's key is (parent global id, successor ordinal in TLC order);
    its fingerprint's owner keeps the smallest key per fingerprint per level
    (the GPU's atomicMin) and replies win/lose;
  * the round's winners, generator-major in shard order, take the next global
    positions and are sent to their block-cyclic owner.
Successors come from the Python oracle (oracle/pyoracle), in TLC order.
"""
import hashlib

import torch.distributed as dist


def owner_of(key, W):
    h = hashlib.blake2b(repr(key).encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") % W


def local_count(P, W, CH, r):
    full, rem = divmod(P, W * CH)
    return full * CH + max(0, min(CH, rem - r * CH))


def gather(obj):
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def sharded_bfs(spec, CH):
    """Run on every rank of an initialised process group; returns the global
    (generated, distinct, depth, levels, status) on every rank."""
    W, r = dist.get_world_size(), dist.get_rank()
    actions = spec.actions()
    init = list(spec.init_states())
    assert len(init) == 1
    table = {}  # this shard's fingerprints: canonical view -> (level, key)
    k0 = spec.canonical(init[0])
    if owner_of(k0, W) == r:
        table[k0] = (1, (0, 0))
    cur = [init[0]] if r == 0 else []  # local states of the current level
    P, base, depth, generated, distinct = 1, 0, 1, 1, 1
    levels = [[1, 1]]
    status = "ok"
    for name, inv in spec.invariants:
        if not inv(init[0]):
            return dict(generated=1, distinct=1, depth=1, levels=levels, status="violation")
    while P:
        level = depth + 1
        rounds = (P + W * CH - 1) // (W * CH)
        nxt = {}  # local index -> state
        GW = gen_lvl = 0
        for c in range(rounds):
            block = cur[c * CH:(c + 1) * CH]
            pbase = base + c * W * CH + r * CH
            cands = []  # (parent local, ordinal, successor, canonical)
            for i, s in enumerate(block):
                k = 0
                for _, fn in actions:
                    for t in fn(s):
                        cands.append((i, k, t, spec.canonical(t)))
                        k += 1
            gen_lvl += sum(gather(len(cands)))
            # records to owners
            out = [[] for _ in range(W)]
            for j, (i, k, t, key) in enumerate(cands):
                out[owner_of(key, W)].append((key, (pbase + i, k), j))
            sent = gather(out)
            recv = [rec for q in range(W) for rec in sent[q][r]]
            for key, kk, _ in recv:
                old = table.get(key)
                if old is None or (old[0] == level and kk < old[1]):
                    table[key] = (level, kk)
            flags = {}  # generator shard -> {candidate index: won}
            for q in range(W):
                flags[q] = {j: table[key] == (level, kk) for key, kk, j in sent[q][r]}
            back = gather(flags)
            won = [any(back[d][r].get(j, False) for d in range(W)) for j in range(len(cands))]
            winners = [cands[j][2] for j in range(len(cands)) if won[j]]  # TLC order: parent, then ordinal
            for t in winners:
                for name, inv in spec.invariants:
                    if not inv(t):
                        status = "violation"
            counts = gather(len(winners))
            go = sum(counts[:r])
            pieces = [[] for _ in range(W)]
            for x, t in enumerate(winners):
                g = GW + go + x
                pieces[(g // CH) % W].append(((g // (W * CH)) * CH + g % CH, t))
            got = gather(pieces)
            for q in range(W):
                for li, t in got[q][r]:
                    nxt[li] = t
            GW += sum(counts)
            if any(s != "ok" for s in gather(status)):
                status = "violation"
                break
        generated += gen_lvl
        distinct += GW
        if GW or gen_lvl:
            levels.append([gen_lvl, GW])
        if GW:
            depth += 1
        n = local_count(GW, W, CH, r)
        assert sorted(nxt) == list(range(n)), "block-cyclic layout has holes"
        cur = [nxt[i] for i in range(n)]
        base += P
        P = GW
        if status != "ok":
            break
    return dict(generated=generated, distinct=distinct, depth=depth, levels=levels, status=status)
