#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + PMC passes) into one JSON/markdown
file under profiles/.  Usage: prof_summary.py OUT.md STATS_DIR [PMC_DIR ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, stats_dir, pmc_dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    lines = ["# rocprofv3 summary: %s" % os.path.basename(out), ""]
    ks = glob.glob(os.path.join(stats_dir, "*kernel_stats.csv"))
    if ks:
        lines += ["## kernel trace --stats (%s)" % os.path.relpath(ks[0]), "",
                  "| kernel | calls | avg ms | min ms | max ms | % |", "|---|---|---|---|---|---|"]
        for r in csv.DictReader(open(ks[0])):
            lines.append("| %s | %s | %.3f | %.3f | %.3f | %s |" % (
                r["Name"], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["MinNs"]) / 1e6,
                float(r["MaxNs"]) / 1e6, r["Percentage"]))
        lines.append("")
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            acc = defaultdict(list)
            for r in csv.DictReader(open(f)):
                acc[(r["Kernel_Name"], r["Counter_Name"])].append(
                    (int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
            lines += ["## PMC %s" % os.path.relpath(f), "",
                      "| kernel | counter | dispatches | value per dispatch (KB for *_SIZE) | ms per dispatch |",
                      "|---|---|---|---|---|"]
            for (k, c), v in sorted(acc.items()):
                byd = {}
                for did, val, ms in v:
                    byd[did] = (val, ms)
                vals = [x[0] for x in byd.values()]
                mss = [x[1] for x in byd.values()]
                lines.append("| %s | %s | %d | %s | %s |" % (
                    k[:60], c, len(byd), " / ".join("%.0f" % x for x in vals), " / ".join("%.2f" % x for x in mss)))
            lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
