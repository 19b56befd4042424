#!/usr/bin/env python3
"""Per-kernel rocprofv3 summary of one bench.py workload -> profiles/.

Inputs (rocprofv3 output directories, each from its own run):
  --trace DIR   rocprofv3 --kernel-trace --stats of `tools/prof_run.py WL S` (1 warmup + S steps)
  --fetch DIR   rocprofv3 --pmc FETCH_SIZE of `tools/prof_run.py WL 1`
  --write DIR   rocprofv3 --pmc WRITE_SIZE of the same command
Outputs: OUT.json (per-kernel launch time and HBM traffic per launch / per read; bench.py
reads traffic_bytes_per_read of the dominant kernel from it) and OUT.md.

Dispatch accounting: every step launches each kernel L times (one per chunk of reads).
The trace holds (W + S + X) * L dispatches per kernel (X: steps after the timed ones --
prof_run.py's host mode runs one more, the HIP-event kernel record): the timed-region average
is over dispatches W*L .. (W+S)*L.  The PMC runs are 1 warmup + 1 step (+ X): their second
step's L dispatches are one step's traffic.  probe_kernel = probe_line_kernel + probe_big_kernel (one probe launch of the library's
timing API brackets both), or the one-kernel probe when the index has no bucket codes/lines.

Units and corrections (MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KiB.  The guide's x2 correction is for 16-B/lane coalesced streaming
reads; these kernels' reads are random 2-64 B gathers, which tools/calib_fetch.hip measured
at one 64-B request each, so the counted values are used as they are."""
import argparse
import glob
import json
import os
import sqlite3
from collections import defaultdict

KERNELS = ("probe_kernel", "probe_line_kernel", "probe_big_kernel", "gather_kernel", "lane_kernel", "vote_kernel",
           "unpack_reads", "compact_records")


def short(name):
    if "lane_pe_kernel" in name:      # bench.py times both lane kernels as "lane_kernel"
        return "lane_kernel"
    for k in KERNELS[1:]:
        if k in name:
            return k
    if "probe_kernel" in name:
        return "probe_kernel"
    return None


def trace(d):
    db = glob.glob(os.path.join(d, "*results.db"))[0]
    c = sqlite3.connect(db)
    per = defaultdict(list)
    for name, s, e in c.execute("select name, start, end from kernels order by start"):
        k = short(name)
        if k:
            per[k].append((int(e) - int(s)) / 1e6)
    stats = {}
    for name, calls, avg, pct in c.execute("select name, total_calls, average, percentage from top_kernels"):
        k = short(name)
        if k:
            stats[k] = {"name": name[:90], "calls": int(calls), "avg_ms": float(avg) / 1e3, "pct": float(pct)}
    return per, stats


def pmc(d, counter):
    db = glob.glob(os.path.join(d, "*results.db"))[0]
    c = sqlite3.connect(db)
    per = defaultdict(list)
    for name, n, v, di in c.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        k = short(name)
        if k and n == counter:
            per[k].append((int(di), float(v)))
    return {k: [v for _, v in sorted(x)] for k, x in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--extra", type=int, default=1, help="steps after the timed ones (prof_run.py host mode: 1)")
    ap.add_argument("--reads", type=int, default=50_000_000, help="reads per step (all chunks)")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--bench-json", help="bench.py line of the traced run (launch_ms to compare)")
    ap.add_argument("--cmd", default="python3 tools/prof_run.py WL STEPS host", help="the profiled command")
    a = ap.parse_args()

    per, stats = trace(a.trace)
    fe, wr = pmc(a.fetch, "FETCH_SIZE"), pmc(a.write, "WRITE_SIZE")
    bench = json.load(open(a.bench_json))["roofline"]["kernels"] if a.bench_json else {}
    res = {"workload": a.workload, "reads_per_step": a.reads, "kernels": {}, "correction":
           "none: random 2-64 B gathers count one 64-B request each (tools/calib_fetch.hip); "
           "the x2 streaming-read correction applies to 16-B/lane streaming reads only"}
    tot_traffic = 0.0
    for k in KERNELS:
        if k not in per:
            continue
        d = per[k]
        L = max(1, len(d) // (a.warmup + a.steps + a.extra))
        timed = d[a.warmup * L:(a.warmup + a.steps) * L]
        f, w = fe.get(k, []), wr.get(k, [])
        pl = max(1, len(f) // (2 + a.extra))      # the PMC runs' launches per step
        nf = pl
        fb = sum(f[pl:2 * pl]) * 1024.0
        wb = sum(w[pl:2 * pl]) * 1024.0
        ent = {"launches_per_step": L, "timed_avg_ms": sum(timed) / max(1, len(timed)),
               "all_dispatch_avg_ms": stats.get(k, {}).get("avg_ms"), "calls": len(d),
               "fetch_bytes_per_read": fb / a.reads, "write_bytes_per_read": wb / a.reads,
               "traffic_bytes_per_read": (fb + wb) / a.reads,
               "traffic_bytes_per_launch": (fb + wb) / max(1, nf),
               "name": stats.get(k, {}).get("name")}
        if k in bench:
            ent["bench_launch_ms"] = bench[k]["launch_ms"]
        res["kernels"][k] = ent
        tot_traffic += fb + wb
    # the library's "probe_kernel" timing kind = line kernel + big-bucket kernel
    if "probe_line_kernel" in res["kernels"] and "probe_kernel" not in res["kernels"]:
        pl, pb = res["kernels"]["probe_line_kernel"], res["kernels"].get("probe_big_kernel")
        comb = dict(pl)
        if pb:
            for f in ("timed_avg_ms", "fetch_bytes_per_read", "write_bytes_per_read", "traffic_bytes_per_read",
                      "traffic_bytes_per_launch"):
                comb[f] = pl[f] + pb[f]
        comb["name"] = "probe_line_kernel + probe_big_kernel"
        comb["all_dispatch_avg_ms"] = None
        res["kernels"]["probe_kernel"] = comb
    res["traffic_bytes_per_read"] = tot_traffic / a.reads
    res["command"] = a.cmd
    json.dump(res, open(a.out + ".json", "w"), indent=1)
    M = ["# rocprofv3 summary: %s (%d timed steps of %d reads)" % (a.workload, a.steps, a.reads), "",
         "Kernel trace: `rocprofv3 --kernel-trace --stats -- %s` (STEPS = %d after %d warmup step).  PMC: "
         "separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs of the same command with STEPS = 1 (no correction: "
         "random gathers, see tools/calib_fetch.hip)." % (a.cmd, a.steps, a.warmup), "",
         "| kernel | launches/step | timed avg ms (trace) | bench.py HIP-event ms | rocprof --stats avg ms (all dispatches) "
         "| FETCH B/read | WRITE B/read | HBM traffic B/read |", "|---|---|---|---|---|---|---|---|"]
    for k, e in res["kernels"].items():
        M.append("| %s | %d | %.3f | %s | %s | %.1f | %.1f | %.1f |" % (
            k, e["launches_per_step"], e["timed_avg_ms"], "%.3f" % e["bench_launch_ms"] if "bench_launch_ms" in e else "-",
            "%.3f" % e["all_dispatch_avg_ms"] if e["all_dispatch_avg_ms"] is not None else "-",
            e["fetch_bytes_per_read"], e["write_bytes_per_read"], e["traffic_bytes_per_read"]))
    M += ["", "Total HBM traffic per read (all kernels of a step): %.1f B" % res["traffic_bytes_per_read"], "",
          "The `--stats` average includes the warmup step; the timed average drops it."]
    open(a.out + ".md", "w").write("\n".join(M) + "\n")
    print("\n".join(M))


if __name__ == "__main__":
    main()
