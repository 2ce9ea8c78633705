#!/usr/bin/env python3
"""Per-dispatch counters of a rocprofv3 --pmc run, in dispatch order:
   pmc_dispatches.py counter_collection.csv [KERNEL_SUBSTRING]
Prints one line per dispatch (kernel, counters).  Used for the k_expand phase
decomposition (RMC_DIAG builds: tools/profile_expand.py launches k_expand 12
times in a row, stopped after each phase, before the level's real launch)."""
import csv
import sys
from collections import OrderedDict

path = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
rows = OrderedDict()
for r in csv.DictReader(open(path)):
    d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    rows.setdefault(d, [k, {}])[1][r["Counter_Name"]] = rows.get(d, [k, {}])[1].get(r["Counter_Name"], 0.0) + \
        float(r["Counter_Value"])
prev = None
run = []
for d in sorted(rows):
    k, c = rows[d]
    if sub and sub not in k:
        continue
    print(d, k[:60], " ".join("%s=%.4g" % (n, v) for n, v in sorted(c.items())))
