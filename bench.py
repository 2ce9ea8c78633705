#!/usr/bin/env python3
"""bench.py — distinct states/s and time-to-exhaust of an exhaustive Raft model
check on MI355X (BASELINE.json metric).

A "step" is one complete exhaustive check of the workload config (BFS from
Init until the frontier is empty), on inputs resident in HBM (the constants
are the input; the frontier, fingerprint set and trace records never leave
the GPU while timed).  `value` = distinct states / seconds-per-check, summed
over ranks.

Multi-GPU: one process per GPU (torch.distributed.run).  N>1 runs ONE check
of the same workload, fingerprint-sharded across the N GPUs (rmc_check_sharded:
RCCL over xGMI); every rank gets the global counts.  Total work
is fixed as N grows ("scaling": "strong"); `value` = distinct states of the
check / seconds per check.  --logical-shards W runs the same sharded protocol
with W shards on one GPU (a measurement of the protocol's overhead).

Run:  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-tlaplus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

# name -> (module, cfg path relative to ROOT, BASELINE config index, description)
WORKLOADS = {
    "raft_cfg": ("Raft", "configs/Raft.cfg", 1,
                 "standard-raft Raft.cfg: 3 servers, Value={v1}, MaxElections=2, MaxRestarts=0"),
    "raft_n3v2e2": ("Raft", "configs/Raft_n3v2e2.cfg", 2,
                    "standard-raft: 3 servers, Value={v1,v2} (log bound 2), MaxElections=2 (term bound 3), "
                    "MaxRestarts=0"),
    "raft_n3v1e3": ("Raft", "configs/Raft_n3v1e3.cfg", 2,
                    "standard-raft: 3 servers, Value={v1}, MaxElections=3, MaxRestarts=0"),
    "raft_n3v2e3": ("Raft", "configs/Raft_n3v2e3.cfg", 2,
                    "standard-raft: 3 servers, Value={v1,v2}, MaxElections=3, MaxRestarts=0"),
}
DEFAULT_WORKLOAD = "raft_n3v2e2"
HBM_PEAK = 8.0e12  # MI355X HBM3E, bytes/s (MI355X_MICROARCH.md chip table)


def algorithmic_bytes(res):
    """Bytes the expand kernel must move per run (SURVEY.md §8d terms it owns):
    every parent state read once (D*S), one fingerprint-set probe per
    successor (G*8), one 12-byte candidate record written per successor."""
    D, G, S = res["distinct"], res["generated"] - 1, res["state_bytes"]
    return D * S + G * 8 + G * 12


def pmc_traffic(workload):
    """Per-launch HBM bytes of k_expand from the committed rocprofv3 --pmc summary
    of this workload (tools/gpu_profile.sh -> profiles/<round>/pmc_summary_<workload>.json),
    priced (2*FETCH_SIZE + WRITE_SIZE) KiB as MI355X_MICROARCH.md prescribes for gfx950."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary_%s.json" % workload)), reverse=True):
        try:
            d = json.load(open(path))
            for k, v in d["kernels"].items():
                if k.startswith("rmc::k_expand") and "traffic_bytes_per_dispatch" in v:
                    return v["traffic_bytes_per_dispatch"], os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def cpu_baseline(module, cfg_path, seconds=20.0):
    """The C oracle (oracle/_build/rmc_oracle, a port) timed on this host for a
    bounded wall budget on the same config; returns distinct states/s."""
    from oracle import run_c
    from oracle.pyoracle.cfg import load_cfg
    exe = run_c.BIN
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    cfg = load_cfg(os.path.join(ROOT, cfg_path))
    threads = max(1, min(16, os.cpu_count() or 1))
    r = run_c.run(module, cfg["constants"], cfg["invariants"], threads=threads,
                  extra=["--max-seconds", str(seconds)])
    return dict(value=r["distinct"] / max(r["seconds"], 1e-9), unit="distinct states/s", cores=threads,
                kind="port",
                sample="C oracle (oracle/cengine) BFS of the same cfg for ~%.0fs wall: %d distinct, %d generated, "
                       "status %s" % (seconds, r["distinct"], r["generated"], r["status"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=os.environ.get("RMC_WORKLOAD", DEFAULT_WORKLOAD))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--logical-shards", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=0, help="parents per k_expand launch (0 = librmc's default)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import torch
    import raftmc

    module, cfg_rel, bcfg, desc = WORKLOADS[args.workload]
    model = raftmc.Model(os.path.join(ROOT, "configs", module + ".tla"), os.path.join(ROOT, cfg_rel))
    if world > 1:
        uid = [raftmc.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        run_check = lambda: model.check_sharded(rank, world, local, uid[0])  # noqa: E731
    elif args.logical_shards:
        run_check = lambda: model.check_logical(args.logical_shards)  # noqa: E731
    else:
        run_check = lambda: model.check(chunk_parents=args.chunk)  # noqa: E731

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    cold = []
    for _ in range(args.warmup):
        t = time.perf_counter()
        run_check()
        cold.append(time.perf_counter() - t)
    barrier()
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        results.append(run_check())
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = results[-1]
    per_step = elapsed / args.steps
    value = res["distinct"] / per_step
    exp_bytes = algorithmic_bytes(res)
    achieved = exp_bytes / (res["expand_ms"] * 1e-3) if res["expand_ms"] > 0 else 0.0
    traffic, traffic_src = pmc_traffic(args.workload)
    if rank == 0:
        line = {
            "metric": "distinct states/sec + time-to-exhaust, standard-raft",
            "value": value,
            "unit": "distinct states/s",
            "n_gpus": world,
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
                       "parallelism": ("fp-sharded x%d (RCCL)" % world) if world > 1 else
                       ("fp-sharded x%d logical shards on 1 GPU" % args.logical_shards if args.logical_shards
                        else "single")},
            "result": {"generated": res["generated"], "distinct": res["distinct"], "depth": res["depth"],
                       "status": res["status"], "time_to_exhaust_s": per_step,
                       "first_check_s": cold[0] if cold else None},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                         "kernel": "k_expand", "launches": res["expand_launches"],
                         "avg_launch_ms": res["expand_ms"] / max(1, res["expand_launches"]),
                         "bytes_per_launch": exp_bytes / max(1, res["expand_launches"])},
            "kernel_ms": {"expand": res["expand_ms"], "mark_scan": res["mark_ms"],
                          "materialize": res["materialize_ms"]},
        }
        # atomic throughput of the fingerprint-set inserts (each
        # successor: one returning CAS per probe + one atomicMin), over k_expand's time
        if res["expand_ms"] > 0:
            line["fpset_inserts"] = {"count": res["generated"] - 1,
                                     "per_s": (res["generated"] - 1) / (res["expand_ms"] * 1e-3),
                                     "atomics_per_insert": ">= 2 (CAS per probe + atomicMin)"}
        if world > 1:
            # exchange volume of the sharded protocol: 16 B (fp, key) records,
            # 1 B win flags, rows + 10 B trace records; the off-GPU fraction is (W-1)/W,
            # point-to-point over xGMI (7 links x ~153 GB/s per MI355X)
            G, D, S = res["generated"] - 1, res["distinct"], res["state_bytes"]
            xb = (G * 17 + D * (S + 10)) * (world - 1) / world
            line["xgmi"] = {"bytes": xb, "per_gpu_GBps": xb / world / per_step / 1e9,
                            "peak_per_gpu_GBps": 7 * 153.0}
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(module, cfg_rel, args.cpu_seconds)
            except Exception as e:  # report, never hide
                line["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
