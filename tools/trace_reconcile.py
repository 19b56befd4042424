#!/usr/bin/env python3
"""One rocprofv3 --kernel-trace of tools/prof_run.py (1 warmup step, STEPS timed steps, 1 HIP-event
record step) -> per-kernel figures checked against the run's own clocks (profiles/r06/...json):

  * per kernel, per launch: the trace's mean duration over the timed steps, beside the HIP-event
    kernel record the same traced process took (svg_set_timing, on each launch's stream) -- the
    two methods measure the same dispatches, so they must agree;
  * per step: the traced step time the process printed, the sum of all kernel durations (over the
    streams: it may exceed the step when kernels overlap) and their busy union (the time any kernel
    ran), which must fit in the step;
  * beside it, untraced runs of the same command (their HIP-event records and step times): the
    tracer's own cost.
Usage: trace_reconcile.py OUT.json --trace DIR --log LOG [--untraced LOG ...] [--label TEXT]"""
import argparse
import glob
import json
import os
import re
import sqlite3


def short(name):
    m = re.match(r"(?:void )?(\w+)", name)
    return m.group(1) if m else name


def step_line(log):
    txt = open(log, errors="replace").read()
    rec = [json.loads(l) for l in txt.splitlines() if l.startswith("{") and "kernel_record" in l]
    m = re.findall(r"([0-9.]+) ms/step, ([0-9.]+) Mreads/s", txt)
    return (rec[-1] if rec else None), (float(m[-1][0]) if m else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--trace", required=True)
    ap.add_argument("--log", required=True)
    ap.add_argument("--untraced", action="append", default=[])
    ap.add_argument("--label", default="")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    db = glob.glob(os.path.join(a.trace, "**", "*results.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    K = [(short(n), int(s), int(e)) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    rec, traced_step = step_line(a.log)
    per_step = rec["kernel_record"]["probe_kernel"]["launches"]
    # steps: the probe kernel launches (probe_line_kernel / probe_kernel) in groups of per_step
    probes = [k for k in K if k[0].startswith("probe_line_kernel") or k[0] == "probe_kernel"]
    nsteps = len(probes) // per_step
    assert nsteps == a.steps + 2, (len(probes), per_step)
    starts = [probes[i * per_step][1] for i in range(nsteps)] + [K[-1][2] + 1]
    timed = []
    for si in range(1, 1 + a.steps):   # the timed steps: not the warmup (0), not the record step (last)
        t0, t1 = starts[si], starts[si + 1]
        ks = [k for k in K if t0 <= k[1] < t1]
        iv = sorted((k[1], k[2]) for k in ks)
        busy, (cs, ce) = 0, iv[0]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        per = {}
        for n, s, e in ks:
            d = per.setdefault(n, [0.0, 0])
            d[0] += (e - s) / 1e6
            d[1] += 1
        timed.append({"span_ms": (max(k[2] for k in ks) - t0) / 1e6, "busy_ms": busy / 1e6,
                      "kernel_sum_ms": sum(v[0] for v in per.values()), "per_kernel": per})
    names = sorted({n for t in timed for n in t["per_kernel"]}, key=lambda n: -sum(t["per_kernel"].get(n, [0])[0] for t in timed))
    kernels = {}
    for n in names:
        ms = sum(t["per_kernel"].get(n, [0, 0])[0] for t in timed)
        nl = sum(t["per_kernel"].get(n, [0, 0])[1] for t in timed)
        kernels[n] = {"ms_per_step": round(ms / a.steps, 3), "launches_per_step": nl // a.steps, "avg_launch_ms": round(ms / nl, 4)}
    # the HIP-event record's kernel names: probe_kernel = every probe launch kind, vote_kernel, lane_kernel
    ev = {k: {"ms_per_step": round(v["ms"], 3), "avg_launch_ms": round(v["ms"] / v["launches"], 4)}
          for k, v in rec["kernel_record"].items()}
    trace_as_record = {
        "probe_kernel": sum(kernels[n]["ms_per_step"] for n in kernels if n.startswith("probe_line_kernel") or n == "probe_kernel"),
        "vote_kernel": sum(kernels[n]["ms_per_step"] for n in kernels if n == "vote_kernel"),
        "lane_kernel": sum(kernels[n]["ms_per_step"] for n in kernels if n in ("lane_kernel", "lane_pe_kernel"))}
    out = {"label": a.label, "trace_dir": a.trace, "traced_log": a.log,
           "traced_step_ms": traced_step,
           "steps": [{k: round(v, 3) for k, v in t.items() if k != "per_kernel"} for t in timed],
           "check_busy_union_fits_step": all(t["busy_ms"] <= traced_step * 1.02 for t in timed),
           "kernels": kernels,
           "hip_events_same_traced_run": ev,
           "trace_vs_hip_events_ms_per_step": {k: [round(trace_as_record[k], 3), ev[k]["ms_per_step"]] for k in trace_as_record if k in ev},
           "untraced": []}
    for lg in a.untraced:
        r, st = step_line(lg)
        out["untraced"].append({"log": lg, "step_ms": st, "options": r.get("options") if r else None,
                                "hip_events": {k: {"ms_per_step": round(v["ms"], 3), "avg_launch_ms": round(v["ms"] / v["launches"], 4)}
                                               for k, v in (r["kernel_record"].items() if r else [])}})
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("traced_step_ms", "steps", "check_busy_union_fits_step", "trace_vs_hip_events_ms_per_step")}))


if __name__ == "__main__":
    main()
