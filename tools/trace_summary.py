#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace database (rocpd SQLite):
trace_summary.py DIR [DIR ...] -- launches, total / average ms per kernel, and the traced span."""
import collections
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
    db = sorted(glob.glob(d + "/**/*.db", recursive=True))[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    agg = collections.defaultdict(list)
    for n, s, e in rows:
        agg[n.split("(")[0].split("<")[0].replace("void ", "")[:40]].append((e - s) / 1e6)
    print("%s: %d dispatches, span %.1f ms" % (d, len(rows), (rows[-1][2] - rows[0][1]) / 1e6))
    for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print("  %-40s n=%5d total=%9.2f ms avg=%.4f ms" % (k, len(v), sum(v), sum(v) / len(v)))
