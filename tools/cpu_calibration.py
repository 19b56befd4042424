#!/usr/bin/env python3
"""CPU baseline calibration: the reference's own voting step vs this
repository's CPU restatement (oracle/svoracle.c, the `cpu_baseline` "port" of bench.py) on
identical reads and the same index, with the same thread count.

Reference: oracle/_ref/subread-align-votetime -- the stock aligner built from /root/reference/src
with oracle/ref_votetime.c answering fetch_next_read_pair: the FASTQ is parsed by the
reference's own parser before the clock starts, and the voting step is timed from there to the
last read of the first pass (run_maybe_threads(STEP_VOTING), core.c:3592: votes, bigtable
writes and the final-run tail of every read).  Its outputs are byte-identical to the stock
binary's (tests/test_dropin.py::test_votetime_harness_matches_stock_reference).  The reference's
own timecost_voting (FASTQ parsing included) is recorded beside it.
Port: svoracle on the same reads held in memory, the vote step only.

Workloads: c3 -- bench.py's C3 genome (3.0 Gbp, 24 contigs, repeat families), full one-block
index (pass --index PREFIX to reuse a prebuilt one), 100 bp SE reads as bench.py simulates them;
c2 -- the 1 Mbp seed-901 genome.  Writes --out (JSON) with reference_over_port.

Usage: tools/cpu_calibration.py [--workload c3|c2] [--index PREFIX] [--reads N] [--threads T] [--out FILE]"""
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
    ap.add_argument("--workload", default="c3", choices=["c3", "c2"])
    ap.add_argument("--index", default="", help="prebuilt reference-format index of the workload's genome")
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04_cpu_calibration.json"))
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--gpu-build", action="store_true",
                    help="write the index files with the GPU builder (svg_index_build_mem, save_prefix): "
                         "same bytes as the CPU builder, minutes faster at 3 Gbp")
    ap.add_argument("--workdir", default="")
    a = ap.parse_args()
    import subread_amd as sa
    from subread_amd.abi import default_params
    from subread_amd.sim import random_genome, simulate_reads, write_fastq, c3_lengths
    from oracle.pyoracle import OracleIndex
    wd = a.workdir or tempfile.mkdtemp(prefix="svg_cal_")
    os.makedirs(wd, exist_ok=True)
    if a.workload == "c3":
        g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
        desc = "C3 genome (3.0 Gbp, 24 contigs, repeat families; bench.py workload c3), full one-block index"
    else:
        g = random_genome([1_000_000], 901)
        desc = "C2 genome (1 Mbp i.i.d., seed 901), full one-block index"
    pre = a.index
    if not pre:
        fa = os.path.join(wd, "genome.fa")
        pre = os.path.join(wd, "full")
        if a.gpu_build:
            ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0, save_prefix=pre)
            ix.close()
        else:
            g.write_fasta(fa)
            sa.build_index(fa, pre, gap=1, force_one_block=True)
    r = simulate_reads(g, a.reads, 100, seed=20261015, sub=0.01, indel=0.001)
    del g
    fq = os.path.join(wd, "reads.fq")
    write_fastq(fq, r)
    ref_bin = os.path.join(ROOT, "oracle", "_ref", "subread-align-votetime")
    ref_t, ref_tc, ref_wall = [], [], []
    for _ in range(a.repeats):
        t = time.perf_counter()
        p = subprocess.run([ref_bin, "-t", "1", "-i", pre, "-r", fq, "-o", os.path.join(wd, "out.sam"), "--SAMoutput",
                            "-T", str(a.threads)], capture_output=True, text=True,
                           env=dict(os.environ, SVG_REF_TIMING="1", SVG_REF_VOTETIME="1"))
        ref_wall.append(time.perf_counter() - t)
        m = re.findall(r"SVG_REF_VOTING_S ([0-9.]+) ([0-9]+)", p.stderr)
        mc = re.findall(r"SVG_REF_TIMECOST_VOTING ([0-9.]+)", p.stderr)
        if p.returncode != 0 or not m or int(m[-1][1]) != a.reads:
            raise SystemExit("reference run failed:\n" + p.stdout[-2000:] + p.stderr[-2000:])
        ref_t.append(float(m[-1][0]))
        if mc:
            ref_tc.append(float(mc[-1]))
        os.remove(os.path.join(wd, "out.sam"))
    oi = OracleIndex(pre)
    prm = default_params()
    port_t = []
    for _ in range(a.repeats):
        t = time.perf_counter()
        oi.vote(prm, r, None, threads=a.threads)
        port_t.append(time.perf_counter() - t)
    oi.close()
    ref_rate = a.reads / min(ref_t)
    port_rate = a.reads / min(port_t)
    model = ""
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    res = {
        "workload": "%d x 100 bp SE reads (1%% substitutions, 0.1%% indels, seed 20261015) vs the %s" % (a.reads, desc),
        "threads": a.threads, "cpu_model": model, "logical_cpus": os.cpu_count(),
        "reference": {"binary": "oracle/_ref/subread-align-votetime (reference sources, gcc -O3, ref_votetime.c)",
                      "voting_step_s": ref_t, "timecost_voting_s": ref_tc, "wall_s": ref_wall, "reads_per_s": ref_rate,
                      "scope": "run_maybe_threads(STEP_VOTING) (core.c:3592) on reads parsed before the clock: "
                               "votes + bigtable writes + the final-run tail; timecost_voting_s also holds the parse"},
        "port": {"library": "oracle/lib/libsvoracle.so (CPU restatement)", "seconds": port_t, "reads_per_s": port_rate,
                 "scope": "vote step on in-memory reads"},
        "reference_over_port": ref_rate / port_rate,
        "summary": "reference voting step %.0f reads/s vs restatement %.0f reads/s, same reads and index (%s), %d threads "
                   "(%s): ratio %.3f" % (ref_rate, port_rate, a.workload.upper(), a.threads, model, ref_rate / port_rate),
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(res["summary"])


if __name__ == "__main__":
    main()
