#!/usr/bin/env python3
"""Fragile junction voting (svg_fragile_batch: core_fragile_junction_voting, core-junction.c:5151-5422,
for subjunc reads > 160 bp) throughput on one GPU, with parity against the oracle restatement and
its CPU time in the same run.  Host reads in, host windows + reported slots out, every kernel and
both copies inside the timed call.

Workload: the C3 genome (3.0 Gbp, 24 contigs, repeat families; bench.py workload c3), index built
in HBM (--gap 1 full one-block, the image the probe reads is the 32-byte bucket code; --gap 3 the
reference's default gapped index, the key-hash image), --reads spliced RNA-seq reads of --len
bases (30% across one GT..AG intron).  Each read gives ~(len - 20) / 40 windows per strand.

  python tools/bench_fragile.py [--gap 1] [--reads 200000] [--len 250] [--steps 3]
-> one JSON line on stdout."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gap", type=int, default=1)
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--len", type=int, default=250)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--check", type=int, default=2000)
    ap.add_argument("--literal", action="store_true", help="option keys_literal: the literal bucket search")
    args = ap.parse_args()
    import torch  # noqa: F401
    import subread_amd as sa
    from subread_amd.abi import default_params, PROGRAM_SUBJUNC
    from subread_amd.sim import c3_lengths, random_genome, simulate_spliced_reads
    from bench import cpu_info
    t0 = time.time()
    genome = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    ix = sa.VoteIndex.build_genome(genome, gap=args.gap, memory_mb=8000, force_one_block=args.gap == 1, device=0)
    reads = simulate_spliced_reads(genome, args.reads, args.len, seed=7007)
    log("[fragile] genome, index and %d reads in %.1fs" % (args.reads, time.time() - t0))
    p = default_params(PROGRAM_SUBJUNC, False)
    sa.set_option("keys_literal", 1 if args.literal else 0)
    res = ix.fragile(p, reads)
    steps = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        res = ix.fragile(p, reads)
        steps.append(time.perf_counter() - ts)
    sec = min(steps)
    w, s = res
    bases = args.reads * args.len
    line = {"metric": "fragile junction voting (svg_fragile_batch), windows/s",
            "value": round(len(w) / sec / 1e6, 3), "unit": "M windows/s", "reads_per_s": round(args.reads / sec, 1),
            "mbases_per_s": round(bases / sec / 1e6, 1), "ms_per_step": round(sec * 1e3, 2),
            "steps_ms": [round(x * 1e3, 2) for x in steps], "windows": int(len(w)), "slots": int(len(s)),
            "junction_windows": int(w["junction"].sum()),
            "probe": "literal bucket search" if args.literal else ("32-byte bucket code" if args.gap == 1 else "key-hash record"),
            "config": {"genome": "C3 3.0 Gbp", "index": "full one-block" if args.gap == 1 else "gapped (gap 3)",
                       "reads": args.reads, "read_len": args.len, "mode": "subjunc SE"}}
    if args.check:
        from oracle.pyoracle import OracleIndex
        oi = OracleIndex(arrays=ix.export())
        k = min(args.check, args.reads)
        sub = reads.slice(0, k)
        gw, gs = ix.fragile(p, sub)
        cpu = cpu_info()
        tc = time.perf_counter()
        ww, ws = oi.fragile(p, sub)
        tc = time.perf_counter() - tc
        same = len(gw) == len(ww) and (gw.view(np.uint8) == ww.view(np.uint8)).all() and len(gs) == len(ws) and \
            (gs.view(np.uint8) == ws.view(np.uint8)).all()
        line["parity_check"] = {"reads": k, "identical": bool(same)}
        line["cpu_restatement"] = {"reads_per_s": round(k / tc, 1), "note": "oracle svo_fragile_batch, one call",
                                   "cpu_model": cpu["model"]}
    print(json.dumps(line), flush=True)
    ix.close()


if __name__ == "__main__":
    main()
