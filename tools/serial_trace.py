#!/usr/bin/env python3
"""Serialised kernel trace of the metric's path -> profiles/<out>.json (bench.py's
roofline.committed.serial_trace reads it).

tools/profile_serial.sh runs `rocprofv3 --kernel-trace --stats -- python3 tools/prof_run.py WL
STEPS host overlap=0`: bench.py's host step with the chunk pipeline's second stream off, so every
kernel of the vote path runs on one stream, one after the other, and the per-launch durations of
a step add up to at most that step's own time under the tracer.  This script takes the trace's
timed-region dispatches (the first `--warmup` steps dropped), the per-step kernel sum and the
step time the traced run printed, and checks sum <= step.
Usage: serial_trace.py TRACE_DIR LOG OUT.json --steps S [--warmup 1]"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_kernels import trace  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("log")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    per, stats = trace(a.trace_dir)
    log = open(a.log).read()
    m = re.search(r"host: (\d+) reads x (\d+) ends, ([0-9.]+) ms/step", log)
    step_ms = float(m.group(3))
    rec = None
    for line in log.splitlines():
        if line.startswith("{") and "kernel_record" in line:
            rec = json.loads(line)
    total = a.steps + a.warmup + (1 if rec else 0)   # + the HIP-event record step
    kern, step_sum = {}, 0.0
    for k, durs in per.items():
        if k == "probe_big_kernel":
            continue
        L = len(durs) // total
        timed = durs[a.warmup * L:(a.warmup + a.steps) * L]
        if k == "probe_line_kernel":      # the library times line + big as one probe launch
            big = per.get("probe_big_kernel", [])
            Lb = len(big) // total
            btimed = big[a.warmup * Lb:(a.warmup + a.steps) * Lb]
            k = "probe_kernel"
            ms = (sum(timed) + sum(btimed)) / max(1, len(timed))
        else:
            ms = sum(timed) / max(1, len(timed))
        kern[k] = {"avg_ms": round(ms, 4), "launches_per_step": L, "per_step_ms": round(ms * L, 3)}
        step_sum += ms * L
    out = {"workload": m.group(0), "kernels": kern, "kernel_sum_per_step_ms": round(step_sum, 3),
           "traced_step_ms": step_ms, "fits": step_sum <= step_ms,
           "hip_event_record": rec,
           "note": "rocprofv3 --kernel-trace of tools/prof_run.py ... host overlap=0 (one stream); "
                   "per-launch averages over the timed steps; probe_kernel = probe_line + probe_big"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({"kernel_sum_per_step_ms": out["kernel_sum_per_step_ms"], "traced_step_ms": step_ms,
                      "fits": out["fits"]}))


if __name__ == "__main__":
    main()
