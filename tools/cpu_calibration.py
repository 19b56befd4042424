#!/usr/bin/env python3
"""CPU baseline calibration: the reference's own voting phase vs this
repository's CPU restatement (oracle/svoracle.c, the `cpu_baseline` "port" of bench.py) on
identical C2 inputs -- 1,000,000 bp i.i.d. genome (seed 901), full one-block index, 100 bp SE
reads (1% substitutions, 0.1% indels, seed 20261015) -- with the same thread count.

Reference: oracle/_ref/subread-align-dump (built from /root/reference/src by oracle/Makefile),
voting time = timecost_voting (core.c:3592-3595; printed by the dump hook, SVG_REF_TIMING=1),
which includes FASTQ parsing and the final-run find_new_indels on top of the vote.  Port:
svoracle on the same reads held in memory.  Writes profiles/r02_cpu_calibration.json with
reference_over_port = (reference reads/s) / (port reads/s).

Usage: tools/cpu_calibration.py [--reads N] [--threads T] [--out FILE]"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"))
    ap.add_argument("--repeats", type=int, default=3)
    a = ap.parse_args()
    import subread_amd as sa
    from subread_amd.abi import default_params
    from subread_amd.sim import random_genome, simulate_reads, write_fastq
    from oracle.pyoracle import OracleIndex
    wd = tempfile.mkdtemp(prefix="svg_cal_")
    g = random_genome([1_000_000], 901)
    fa = os.path.join(wd, "c2.fa")
    g.write_fasta(fa)
    pre = os.path.join(wd, "c2_full")
    sa.build_index(fa, pre, gap=1, force_one_block=True)
    r = simulate_reads(g, a.reads, 100, seed=20261015, sub=0.01, indel=0.001)
    fq = os.path.join(wd, "reads.fq")
    write_fastq(fq, r)
    ref_bin = os.path.join(ROOT, "oracle", "_ref", "subread-align-dump")
    ref_t, ref_wall = [], []
    for _ in range(a.repeats):
        t = time.perf_counter()
        p = subprocess.run([ref_bin, "-t", "1", "-i", pre, "-r", fq, "-o", os.path.join(wd, "out.sam"), "--SAMoutput",
                            "-T", str(a.threads)], capture_output=True, text=True, env=dict(os.environ, SVG_REF_TIMING="1"))
        ref_wall.append(time.perf_counter() - t)
        m = re.findall(r"SVG_REF_TIMECOST_VOTING ([0-9.]+)", p.stderr)
        if p.returncode != 0 or not m:
            raise SystemExit("reference run failed:\n" + p.stdout[-2000:] + p.stderr[-2000:])
        ref_t.append(float(m[-1]))
    oi = OracleIndex(pre)
    prm = default_params()
    port_t = []
    for _ in range(a.repeats):
        t = time.perf_counter()
        oi.vote(prm, r, None, threads=a.threads)
        port_t.append(time.perf_counter() - t)
    ref_rate = a.reads / min(ref_t)
    port_rate = a.reads / min(port_t)
    model = ""
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    res = {
        "workload": "C2: %d x 100 bp SE reads vs 1 Mbp i.i.d. genome (seed 901), full one-block index" % a.reads,
        "threads": a.threads, "cpu_model": model, "logical_cpus": os.cpu_count(),
        "reference": {"binary": "oracle/_ref/subread-align-dump (reference sources, gcc -O3)",
                      "timecost_voting_s": ref_t, "wall_s": ref_wall, "reads_per_s": ref_rate,
                      "scope": "timecost_voting (core.c:3592-3595): FASTQ parsing + voting + final-run find_new_indels"},
        "port": {"library": "oracle/lib/libsvoracle.so (CPU restatement)", "seconds": port_t, "reads_per_s": port_rate,
                 "scope": "vote step on in-memory reads"},
        "reference_over_port": ref_rate / port_rate,
        "summary": "reference %.0f reads/s vs restatement %.0f reads/s on identical C2 reads, %d threads (%s): "
                   "ratio %.3f" % (ref_rate, port_rate, a.threads, model, ref_rate / port_rate),
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(res["summary"])


if __name__ == "__main__":
    main()
