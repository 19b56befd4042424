#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run (results.db): per-kernel and
per-copy time inside the last WINDOW seconds, GPU busy time (union of kernels), and the idle gaps
between kernels -- to see what a pipeline leaves on the table.  Usage: timeline.py DIR [WINDOW_S]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

d = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
db = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)[0]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables:", tabs)
for t in tabs:
    if "kernel" in t or "memory" in t or "copy" in t:
        cols = [r[1] for r in c.execute("pragma table_info('%s')" % t)]
        print(t, cols)
K = list(c.execute("select name, start, end from kernels order by start"))
M = []
for t in tabs:
    if t in ("memory_copies", "memory_copy"):
        cols = [r[1] for r in c.execute("pragma table_info('%s')" % t)]
        nm = "name" if "name" in cols else cols[0]
        sz = "size" if "size" in cols else None
        q = "select %s, start, end%s from %s order by start" % (nm, ", " + sz if sz else "", t)
        M = list(c.execute(q))
t_end = max(int(e) for _, _, e in K)
t0 = t_end - win * 1e9
kt = defaultdict(lambda: [0, 0.0])
iv = []
for n, s, e in K:
    s, e = int(s), int(e)
    if s < t0:
        continue
    k = n.split("(")[0].split("<")[0][-40:]
    kt[k][0] += 1
    kt[k][1] += (e - s) / 1e6
    iv.append((s, e))
iv.sort()
busy, cur_s, cur_e, gaps = 0, None, None, []
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
span = (iv[-1][1] - iv[0][0]) if iv else 0
print("window %.3f s: kernels busy %.1f ms of %.1f ms span; %d gaps, %.1f ms idle, largest %s us" % (
    win, busy / 1e6, span / 1e6, len(gaps), sum(gaps) / 1e6, sorted(gaps)[-5:] and [round(g / 1e3) for g in sorted(gaps)[-5:]]))
for k, (cnt, ms) in sorted(kt.items(), key=lambda x: -x[1][1]):
    print("  %-40s %5d launches %8.2f ms" % (k, cnt, ms))
mt = defaultdict(lambda: [0, 0.0, 0])
for row in M:
    n, s, e = row[0], int(row[1]), int(row[2])
    if s < t0:
        continue
    mt[str(n)][0] += 1
    mt[str(n)][1] += (e - s) / 1e6
    if len(row) > 3 and row[3] is not None:
        mt[str(n)][2] += int(row[3])
for k, (cnt, ms, b) in mt.items():
    print("  copy %-30s %5d %8.2f ms %10.1f MB" % (k, cnt, ms, b / 1e6))
