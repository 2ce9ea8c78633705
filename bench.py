#!/usr/bin/env python3
"""bench.py — distinct states/s and time-to-exhaust of an exhaustive Raft model
check on MI355X (BASELINE.json metric).

A "step" is one complete exhaustive check of the workload config (BFS from
Init until the frontier is empty), on inputs resident in HBM (the constants
are the input; the frontier, fingerprint set and trace records never leave
the GPU while timed).  `value` = distinct states / seconds-per-check, summed
over ranks.

Multi-GPU: N>1 runs ONE check of the same workload, fingerprint-sharded
across the N GPUs; every shard gets the global counts.  Under
torch.distributed.run (one process per GPU) it is rmc_check_sharded over RCCL
and the world size must equal --gpus; started plainly, `--gpus N` is the
library's own front door, rmc_check with n_gpus = N (one host thread per GPU,
in-process RCCL) -- which fails, and bench.py with it, when fewer than N GPUs
are visible.  Total work is fixed as N grows ("scaling": "strong"); `value` =
distinct states of the check / seconds per check.  --logical-shards W runs the
same sharded protocol with W shards on one GPU (the protocol's overhead).

Run:  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-tlaplus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

# name -> (module, cfg path relative to ROOT, BASELINE config label, description)
WORKLOADS = {
    "raft_cfg": ("Raft", "configs/Raft.cfg", "1",
                 "standard-raft Raft.cfg: 3 servers, Value={v1}, MaxElections=2, MaxRestarts=0"),
    "raft_n3v2e2": ("Raft", "configs/Raft_n3v2e2.cfg",
                    "2 ladder, rung below config 2 (config 2 itself, MaxElections=3, does not exhaust on one GPU: "
                    "levels paged to host memory, it stops at depth 29, 2.03e9 distinct, on the 245 GiB host-page "
                    "limit: profiles/r03/ladder_Raft_n3v2e3_pin4.txt)",
                    "standard-raft: 3 servers, Value={v1,v2} (logs <= 2 entries), MaxElections=2 (terms <= 3), "
                    "MaxRestarts=0; the largest config-2 rung that exhausts on one MI355X"),
    "raft_n3v1e3": ("Raft", "configs/Raft_n3v1e3.cfg", "2 ladder (Value={v1})",
                    "standard-raft: 3 servers, Value={v1}, MaxElections=3 (terms <= 4), MaxRestarts=0"),
    "raft_n3v2e3": ("Raft", "configs/Raft_n3v2e3.cfg", "2",
                    "standard-raft: 3 servers, Value={v1,v2}, MaxElections=3 (terms <= 4), MaxRestarts=0"),
    "kraft_cfg": ("KRaft", "configs/KRaft.cfg", "SURVEY 8f rank 3 (KRaft)",
                  "KRaft.cfg (pull-raft/KRaft.cfg): 3 servers, Value={v1}, MaxElections=2, MaxRestarts=0"),
    "kraft_n3v2e2": ("KRaft", "configs/KRaft_n3v2e2.cfg", "SURVEY 8f rank 3 (KRaft)",
                     "KRaft: 3 servers, Value={v1,v2}, MaxElections=2, MaxRestarts=0"),
}
DEFAULT_WORKLOAD = "raft_n3v2e2"
HBM_PEAK = 8.0e12  # MI355X HBM3E, bytes/s (MI355X_MICROARCH.md chip table)


def algorithmic_bytes(res):
    """B = D*S (read each parent once) + G*8 (fp probe) + D*8 (fp
    store) + D*S (write new state) + D*12 (trace record), for the whole check."""
    D, G, S = res["distinct"], res["generated"] - 1, res["state_bytes"]
    return 2 * D * S + 8 * G + 20 * D


def pmc_summary(workload):
    """The committed rocprofv3 --pmc summary of this workload (newest round first):
    per-kernel HBM traffic per dispatch, priced as tools/pmc_summary.py states."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary_%s.json" % workload)), reverse=True):
        try:
            return json.load(open(path)), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def host_cores():
    """CPU threads this process may use: its affinity set, capped by the box's
    OMP_NUM_THREADS share when set (the GPU box exports 16), and the CPU model."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit():
        n = min(n, int(cap))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return max(1, n), model


def cpu_baseline(module, cfg_path, seconds=15.0):
    """BASELINE.md's CPU baseline: the build's own multi-threaded C++ BFS
    (rmc_check_cpu -- same packed layout, lowered actions, fingerprint and
    first-in-TLC-order rule as the GPU path) on this host's cores, on the same
    config for a bounded wall budget (it stops at the first level boundary past
    it); rate = distinct states / seconds of the levels it completed."""
    import raftmc
    cores, model = host_cores()
    m = raftmc.Model(module=module, cfg_path=os.path.join(ROOT, cfg_path))
    r = m.check_cpu(workers=cores, time_limit=seconds)
    out = dict(value=r["distinct"] / max(r["seconds"], 1e-9), unit="distinct states/s", cores=cores,
               kind="port", cpu_model=model,
               sample="librmc CPU engine (rmc_check_cpu, %d threads) on the same cfg until the first level boundary "
                      "past %.0f s: %d levels, %d distinct, %d generated in %.1f s (status %s)"
                      % (cores, seconds, r["depth"], r["distinct"], r["generated"], r["seconds"], r["status"]))
    # the whole check on a CPU, for time-to-exhaust: the C oracle's committed
    # run over this cfg (not timed here; measured in the build container)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "oracle_*.json")), reverse=True):
        try:
            o = json.load(open(path))
        except (OSError, ValueError):
            continue
        if o.get("cfg_path") == cfg_path and o.get("status") == "ok":
            out["full_check"] = dict(seconds=o["seconds"], threads=o["threads"], distinct=o["distinct"],
                                     source=os.path.relpath(path, ROOT),
                                     what="C oracle (exact canonical forms) over the whole check, in the build "
                                          "container, not on this host")
            break
    # ... and the CPU engine's own whole check on the GPU box's host (same
    # threads as the sample above), for a same-host time-to-exhaust
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "cpu_full_*.json")), reverse=True):
        try:
            o = json.load(open(path))
        except (OSError, ValueError):
            continue
        if o.get("cfg_path") == cfg_path and o.get("status") == "ok":
            out["full_check_same_host"] = dict(seconds=o["seconds"], threads=o["threads"], distinct=o["distinct"],
                                               source=os.path.relpath(path, ROOT),
                                               what="the CPU engine over the whole check on the GPU box's host "
                                                    "(%s; not timed here)" % o.get("host", "?"))
            break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=os.environ.get("RMC_WORKLOAD", DEFAULT_WORKLOAD))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--logical-shards", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=0, help="parents per k_expand launch (0 = librmc's default)")
    ap.add_argument("--fp-bits", type=int, default=64, choices=(64, 128),
                    help="fingerprint width (128: confirms the 64-bit counts are collision-free)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        print("bench.py: --gpus %d but the launcher started %d ranks" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    if args.gpus < 1:
        print("bench.py: --gpus must be at least 1", file=sys.stderr)
        sys.exit(2)
    inproc = world == 1 and args.gpus > 1  # the library's n_gpus front door, one host thread per GPU
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import torch
    import raftmc

    module, cfg_rel, bcfg, desc = WORKLOADS[args.workload]
    model = raftmc.Model(module=module, cfg_path=os.path.join(ROOT, cfg_rel))
    if world > 1:
        uid = [raftmc.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        run_check = lambda: model.check_sharded(rank, world, local, uid[0])  # noqa: E731
    elif inproc:
        run_check = lambda: model.check(n_gpus=args.gpus, chunk_parents=args.chunk)  # noqa: E731
    elif args.logical_shards:
        run_check = lambda: model.check_logical(args.logical_shards)  # noqa: E731
    else:
        run_check = lambda: model.check(chunk_parents=args.chunk, fp_bits=args.fp_bits)  # noqa: E731

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    cold = []
    cold_phases = None
    for _ in range(args.warmup):
        t = time.perf_counter()
        try:
            run_check()
        except raftmc.RaftmcError as e:  # e.g. more GPUs asked for than visible: never a silent 1-GPU line
            print("bench.py: %s" % e, file=sys.stderr)
            sys.exit(1)
        cold.append(time.perf_counter() - t)
        if cold_phases is None and world == 1 and not inproc and not args.logical_shards:
            cold_phases = model.phases()
            cold_phases["bench_wall"] = cold[-1]
    barrier()
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        try:
            results.append(run_check())
        except raftmc.RaftmcError as e:
            print("bench.py: %s" % e, file=sys.stderr)
            sys.exit(1)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = results[-1]
    per_step = elapsed / args.steps
    value = res["distinct"] / per_step
    B = algorithmic_bytes(res)
    launches = max(1, res["expand_launches"])
    G, D, S = res["generated"] - 1, res["distinct"], res["state_bytes"]
    pmc, pmc_src = pmc_summary(args.workload)
    kpmc = {}
    if pmc and world == 1 and not args.logical_shards:  # the summary profiles the single-shard kernels
        for k, v in pmc.get("kernels", {}).items():
            for short in ("k_expand", "k_mark", "k_materialize"):
                if k.startswith("rmc::" + short) and "traffic_bytes_per_dispatch" in v:
                    kpmc[short] = v["traffic_bytes_per_dispatch"]
    # per-kernel shares of SURVEY §8d's bytes, per launch (every kernel runs
    # once per chunk): k_expand reads the parents and probes / stores the
    # fingerprints; k_materialize writes the new states and trace records
    kern = {}
    for name, bytes_check, ms in (("k_expand", D * S + 8 * G + 8 * D, res["expand_ms"]),
                                  ("k_materialize", D * S + 12 * D, res["materialize_ms"])):
        avg = ms / launches
        ach = bytes_check / launches / (avg * 1e-3) if avg > 0 else 0.0
        kern[name] = {"bytes_per_launch": bytes_check / launches, "avg_launch_ms": avg, "achieved": ach / 1e9,
                      "frac": ach / HBM_PEAK, "traffic": kpmc.get(name)}
    # The peak is HBM's (no MFMA: integer work), but while the check runs far
    # below it the kernels are bound by memory LATENCY -- k_expand's waves wait
    # on dependent round trips (row staging, the tile's reservation atomic, the
    # probe, the CAS) most of their cycles (PMC SQ_WAIT_ANY / SQ_WAVE_CYCLES).
    frac_check = B / per_step / HBM_PEAK
    wait_share = None
    if pmc:
        for k, v in pmc.get("kernels", {}).items():
            if k.startswith("rmc::k_expand") and v.get("SQ_WAVE_CYCLES_per_dispatch"):
                wait_share = v["SQ_WAIT_ANY_per_dispatch"] / v["SQ_WAVE_CYCLES_per_dispatch"]
    bound = "latency" if frac_check < 0.2 else "hbm"
    bound_detail = ("k_expand waves wait %.0f%% of their cycles (PMC SQ_WAIT_ANY / SQ_WAVE_CYCLES, %s)"
                    % (100 * wait_share, pmc_src)) if wait_share is not None else None
    if rank == 0:
        line = {
            "metric": "distinct states/sec + time-to-exhaust, " +
                      {"Raft": "standard-raft", "KRaft": "KRaft"}.get(module, module),
            "value": value,
            "unit": "distinct states/s",
            "n_gpus": world if world > 1 else args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: the model constants are the input (no dataset)",
            "config": {"workload": args.workload, "baseline_config": bcfg, "description": desc,
                       "spec": module, "cfg": cfg_rel,
                       "parallelism": ("fp-sharded x%d (RCCL, one process per GPU)" % world) if world > 1 else
                       ("fp-sharded x%d (n_gpus: one host thread per GPU, in-process RCCL)" % args.gpus) if inproc else
                       ("fp-sharded x%d logical shards on 1 GPU" % args.logical_shards if args.logical_shards
                        else "single")},
            "result": {"generated": res["generated"], "distinct": res["distinct"], "depth": res["depth"],
                       "status": res["status"], "time_to_exhaust_s": per_step,
                       "first_check_s": cold[0] if cold else None,
                       "first_check_phases": cold_phases,
                       "first_check_note": "the warm-up check of this process, by phase (rmc_check_phases, seconds): "
                                           "hip_init = runtime + device context, buffers = arena allocation and VMM "
                                           "maps, launch_enqueue = host time in launch calls (code-object loading on "
                                           "a fresh process), table_growth (.allocate = hipMalloc of each doubled "
                                           "set, the driver's own time; .fill; .rehash) / buffer_growth / widening, "
                                           "kernels = summed device time",
                       "hidden_var_collisions": res["hidden_var_collisions"],
                       "fpset_slots": res["hash_capacity"], "state_bytes": S, "fp_bits": args.fp_bits},
            # achieved = B / t_wall with B = 2DS + 8G + 20D per check;
            # the dominant kernels' own shares per launch under "kernels"
            # (HIP-event launch times inside librmc)
            "roofline": {"bound": bound, "bound_detail": bound_detail, "peak_of": "hbm",
                         "achieved": B / per_step / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": B / per_step / HBM_PEAK,
                         "traffic": sum(kpmc.values()) * launches if len(kpmc) == 3 else None,
                         "traffic_unit": "HBM bytes per check (PMC: k_expand + k_mark + k_materialize)",
                         "traffic_source": pmc_src if kpmc else None,
                         "formula": "B = 2*D*S + 8*G + 20*D per check (SURVEY.md 8d) over the check's wall time",
                         "bytes_per_check": B, "kernel": "k_expand", "launches": launches, "kernels": kern,
                         "candidate_bytes_per_check": G * (8 + 4 + 2)},
            "kernel_ms": {"expand": res["expand_ms"], "mark_scan": res["mark_ms"],
                          "materialize": res["materialize_ms"]},
        }
        # atomic throughput of the fingerprint-set inserts over k_expand's time
        if res["expand_ms"] > 0:
            line["fpset_inserts"] = {"count": G, "per_s": G / (res["expand_ms"] * 1e-3),
                                     "atomics": "duplicates of earlier levels: none (plain loads); new "
                                                "fingerprints: CAS + atomicMin; same-level duplicates: atomicMin"}
        if world > 1 or inproc:
            nw = args.gpus
            # exchange volume of the sharded protocol: 16 B (fp, key) records,
            # 1 B win flags, rows + 10 B trace records; the off-GPU fraction is (W-1)/W,
            # point-to-point over xGMI (7 links x ~153 GB/s per MI355X)
            G, D, S = res["generated"] - 1, res["distinct"], res["state_bytes"]
            xb = (G * 17 + D * (S + 10)) * (nw - 1) / nw
            line["xgmi"] = {"bytes": xb, "per_gpu_GBps": xb / nw / per_step / 1e9,
                            "peak_per_gpu_GBps": 7 * 153.0}
        if world == 1 and not inproc and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(module, cfg_rel, args.cpu_seconds)
            except Exception as e:  # report, never hide
                line["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
