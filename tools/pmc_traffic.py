#!/usr/bin/env python3
"""HBM traffic of the vote kernel from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Usage:
  pmc_traffic.py OUT.json --fetch DIR --write DIR [--calib-fetch DIR --calib-write DIR]
                 [--stats DIR] [--workload c3] [--md OUT.md]

Each DIR is a rocprofv3 output directory (run_results.db, or *_counter_collection.csv).
The vote kernel's first dispatch is the timed-configuration launch (bench.py
--steps 1 --warmup 0); later dispatches are bench.py's stats pass and are
reported but not used.

Units and corrections (MI355X_MICROARCH.md, "HBM" and "rocprofv3 PMC slots"):
FETCH_SIZE and WRITE_SIZE are in KB (1024 B).  The guide's x2 correction holds
for 16-B/lane coalesced streaming reads; for other widths it says to calibrate
on our own access pattern.  tools/calib_fetch.hip does that: the resulting
bytes-per-access figures are written next to the traffic so the reader can see
which correction applies.  The vote kernel's reads are random 2-64 B gathers
(calibrated at one 64-B request each, no x2), so traffic = FETCH_SIZE + WRITE_SIZE
as counted.
"""
import argparse
import csv
import glob
import json
import os
import sqlite3


def rows(d):
    """(kernel, counter, value, dispatch_id, duration_ns) from a rocprofv3 output dir."""
    out = []
    dbs = glob.glob(os.path.join(d, "*results.db"))
    if dbs:
        c = sqlite3.connect(dbs[0])
        for k, n, v, di, s, e in c.execute(
                "select kernel_name, counter_name, value, dispatch_id, start, end from counters_collection"):
            out.append((k, n, float(v), int(di), int(e) - int(s)))
        return out
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            out.append((r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), int(r["Dispatch_Id"]),
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def kernel_stats(d):
    dbs = glob.glob(os.path.join(d, "*results.db"))
    res = []
    if dbs:
        c = sqlite3.connect(dbs[0])
        for name, calls, tot, avg, pct in c.execute("select name, total_calls, total_duration, average, percentage "
                                                    "from top_kernels"):
            res.append((name, int(calls), float(avg) / 1e3, float(pct)))   # top_kernels is in us
        # per-dispatch durations of the vote kernel
        durs = [(int(e) - int(s)) / 1e6 for (s, e) in c.execute(
            "select start, end from kernels where name like 'void vote_kernel%' or name like 'void probe_kernel%' "
            "order by start")]
        return res, durs
    for f in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            res.append((r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
    return res, []


def per_dispatch(rs, prefix, counter):
    v = sorted((di, val, dur) for k, n, val, di, dur in rs if k.startswith(prefix) and n == counter)
    return v


def step_total(rs, counter, n_steps_dispatches):
    """Sum of a counter over the probe_kernel + vote_kernel dispatches of the first (timed)
    bench step: the step's dispatches are the first n_steps_dispatches of each kernel."""
    tot = 0.0
    for kern in ("void probe_kernel", "void vote_kernel"):
        d = per_dispatch(rs, kern, counter)
        tot += sum(x[1] for x in d[:n_steps_dispatches])
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("--stats")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--reads", type=int, default=50_000_000)
    ap.add_argument("--md")
    a = ap.parse_args()

    kern = "void vote_kernel"
    f = per_dispatch(rows(a.fetch), kern, "FETCH_SIZE")
    w = per_dispatch(rows(a.write), kern, "WRITE_SIZE")
    assert f and w, "no vote_kernel dispatches in the PMC passes"
    kname = "probe_kernel + " + [k for k, n, *_ in rows(a.fetch) if k.startswith(kern)][0]
    # bench.py --steps 1 --warmup 0 runs the timed step, then the stats pass: half the
    # dispatches of each kernel belong to the timed step
    nd = max(1, len(f) // 2)
    fetch_b = step_total(rows(a.fetch), "FETCH_SIZE", nd) * 1024.0
    write_b = step_total(rows(a.write), "WRITE_SIZE", nd) * 1024.0
    res = {"workload": a.workload, "kernel": kname, "reads_per_launch": a.reads,
           "fetch_bytes": fetch_b, "write_bytes": write_b, "traffic_bytes": fetch_b + write_b,
           "traffic_bytes_per_read": (fetch_b + write_b) / a.reads,
           "fetch_bytes_per_read": fetch_b / a.reads, "write_bytes_per_read": write_b / a.reads,
           "pmc_dispatch_ms": f[0][2] / 1e6,
           "other_dispatches_fetch_kb": [x[1] for x in f[1:]], "other_dispatches_write_kb": [x[1] for x in w[1:]],
           "correction": "none: random 2-64 B gathers count one 64-B request each (tools/calib_fetch.hip); "
                         "the x2 streaming-read correction does not apply"}
    if a.calib_fetch and a.calib_write:
        cf, cw = rows(a.calib_fetch), rows(a.calib_write)
        M = 16 << 20
        cal = {}
        for k, n, v, di, dur in cf:
            if k.startswith("k_stream16"):
                cal["stream16_fetch_over_true"] = v * 1024 / (1 << 30)
            elif "k_gather<unsigned int, 1>" in k:
                cal["gather_u32_fetch_B_per_access"] = v * 1024 / M
            elif "k_gather<short, 1>" in k:
                cal["gather_i16_fetch_B_per_access"] = v * 1024 / M
            elif "k_gather<unsigned int, 8>" in k:
                cal["gather_32B_run_fetch_B_per_access"] = v * 1024 / M
        for k, n, v, di, dur in cw:
            if k.startswith("k_store4"):
                cal["store_u32_write_B_per_access"] = v * 1024 / M
        res["calibration"] = cal
    if a.stats:
        ks, durs = kernel_stats(a.stats)
        res["kernel_trace_vote_ms_per_dispatch"] = durs
        res["kernel_stats"] = [{"kernel": k[:80], "calls": c, "avg_ms": m, "pct": p} for k, c, m, p in ks[:8]]
    json.dump(res, open(a.out, "w"), indent=1)
    if a.md:
        L = ["# rocprofv3 summary — %s (%s)" % (a.workload, kname), ""]
        if a.stats:
            L += ["## `rocprofv3 --kernel-trace --stats` (bench.py --steps 3 --warmup 1)", "",
                  "| kernel | calls | avg ms | % |", "|---|---|---|---|"]
            for k, c, m, p in ks[:8]:
                L.append("| %s | %d | %.3f | %.1f |" % (k[:70], c, m, p))
            L += ["", "probe_kernel / vote_kernel per-dispatch ms in launch order (warmup step, 3 timed steps, "
                  "stats pass; each step = one probe_kernel + vote_kernel pair per chunk of reads): " +
                  ", ".join("%.1f" % x for x in durs), ""]
        L += ["## PMC (separate passes, `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE`, bench.py --steps 1 --warmup 0)", "",
              "| | bytes per launch | bytes per read |", "|---|---|---|",
              "| FETCH_SIZE | %.3e | %.1f |" % (fetch_b, fetch_b / a.reads),
              "| WRITE_SIZE | %.3e | %.1f |" % (write_b, write_b / a.reads),
              "| traffic | %.3e | %.1f |" % (fetch_b + write_b, (fetch_b + write_b) / a.reads), ""]
        if "calibration" in res:
            L += ["## Calibration (tools/calib_fetch.hip, 4 GiB buffer, 16M accesses per kernel)", ""]
            for k, v in res["calibration"].items():
                L.append("* %s = %.3f" % (k, v))
            L.append("")
        L.append("Correction applied: " + res["correction"])
        open(a.md, "w").write("\n".join(L) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
