#!/usr/bin/env python3
"""Per-kernel and per-copy totals from a rocprofv3 rocpd database (the
default output format): python3 tools/rocpd_summary.py DIR/run_results.db"""
import sqlite3
import sys

for path in sys.argv[1:]:
    c = sqlite3.connect(path)
    print(path)
    for name, n, ms in c.execute("select name, count(*), sum(end-start)/1e6 from kernels group by name order by 3 desc"):
        print("  K %-70s %7d %10.1f ms" % (name[:70], n, ms))
    for name, n, ms, gb in c.execute("select name, count(*), sum(end-start)/1e6, sum(size)/1e9 from memory_copies group by name"):
        print("  C %-70s %7d %10.1f ms %8.3f GB" % (name, n, ms, gb))
    t = c.execute("select min(start), max(end) from kernels").fetchone()
    print("  span %.1f ms" % ((t[1] - t[0]) / 1e6))
