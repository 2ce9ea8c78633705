#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + --pmc passes) per kernel.

usage: pmc_summary.py OUT.json --stats run_kernel_stats.csv --pmc pass1_counter_collection.csv [--pmc ...]
       [--workload NAME]

Per kernel (template arguments stripped): dispatches, mean duration, and the
mean per-dispatch value of every counter found.  HBM traffic per dispatch
(FETCH_SIZE and WRITE_SIZE are in KiB):
    traffic_bytes = (FETCH_SIZE + WRITE_SIZE) * 1024             (raw counters)
    traffic_bytes_streaming = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
The microarch guide calibrates only wide coalesced streaming reads (FETCH_SIZE
= half their bytes: the second figure).  Our own calibration
(rmc_fpset_bench -calib, profiles/r02/pmc_calibration.json) of the random
accesses the fingerprint set makes: one random 16 B read counts 64 B of
FETCH_SIZE; one random 8 B atomicMin counts 32 B of WRITE_SIZE and no
FETCH_SIZE.  The BFS kernels mix streamed rows with random probes, so the raw
sum is reported as the traffic and the streaming-corrected one beside it.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    name = name.strip('"')
    m = re.match(r"(?:void )?([\w:]+?)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--stats")
    ap.add_argument("--pmc", action="append", default=[])
    ap.add_argument("--workload", default="")
    a = ap.parse_args()
    res = {"workload": a.workload, "kernels": {}}
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            k = short(r["Name"])
            res["kernels"].setdefault(k, {}).update(
                calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), total_ns=float(r["TotalDurationNs"]),
                percent=float(r["Percentage"]))
    for path in a.pmc:
        sums = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            c = r["Counter_Name"]
            sums[k][c] += float(r["Counter_Value"])
            disp[(k, c)].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        for k, cs in sums.items():
            d = res["kernels"].setdefault(k, {})
            for c, v in cs.items():
                n = max(1, len(disp[(k, c)]))
                d["pmc_dispatches"] = n
                d[c + "_per_dispatch"] = v / n
    for k, d in res["kernels"].items():
        if "FETCH_SIZE_per_dispatch" in d and "WRITE_SIZE_per_dispatch" in d:
            d["traffic_bytes_per_dispatch"] = (d["FETCH_SIZE_per_dispatch"] + d["WRITE_SIZE_per_dispatch"]) * 1024
            d["traffic_bytes_streaming_per_dispatch"] = (2 * d["FETCH_SIZE_per_dispatch"] +
                                                         d["WRITE_SIZE_per_dispatch"]) * 1024
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: {x: v for x, v in d.items() if x in ("calls", "avg_ns", "traffic_bytes_per_dispatch")}
                      for k, d in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
