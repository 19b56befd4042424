#!/usr/bin/env python3
"""sublong's voting step (svg_long_vote_batch) throughput on one GPU, with parity and a CPU
baseline in the same run.  Not bench.py's metric (that is the short-read vote path): this is
the f4 row's long-read reuse, measured the same way -- host reads in, host results out
(H2D of the text, every kernel, D2H of the slots and orders inside the timed call).

Workload: the C3 genome (3.0 Gbp, 24 contigs, injected repeat families; bench.py workload c3),
index built in HBM (--gap 1: full one-block; --gap 3: the reference's default gapped index);
--reads simulated ONT-like long reads (log-normal lengths around --mean-len, 3% substitutions,
2% insertions, 2% deletions).  Parity: the first --check reads against the oracle restatement
(oracle/svoracle.c, pinned to the reference's own longread-one code by tests/test_sublong.py);
CPU baseline: that restatement on --cpu-reads reads with the process's usable CPUs.

  python tools/bench_long.py [--gap 1] [--reads 20000] [--mean-len 8000] [--steps 3]
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
    ap.add_argument("--reads", type=int, default=20000)
    ap.add_argument("--mean-len", type=int, default=8000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--check", type=int, default=400)
    ap.add_argument("--cpu-reads", type=int, default=2000)
    ap.add_argument("--genome", default="c3", choices=["c3", "small"])
    args = ap.parse_args()
    import torch  # noqa: F401  (device plumbing only)
    import subread_amd as sa
    from subread_amd.sim import c3_lengths, random_genome, simulate_long_reads
    from bench import cpu_info
    t0 = time.time()
    if args.genome == "c3":
        genome = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    else:
        genome = random_genome([20_000_000, 10_000_000], 77, repeats=(20_000, 300, 40, 0.12))
    log("[long] genome %.3f Gbp in %.1fs" % (genome.length / 1e9, time.time() - t0))
    t1 = time.time()
    ix = sa.VoteIndex.build_genome(genome, gap=args.gap, memory_mb=8000, force_one_block=args.gap == 1, device=0)
    log("[long] index in HBM (%.1f GB) in %.1fs" % (ix.info.device_bytes / 1e9, time.time() - t1))
    t1 = time.time()
    reads = simulate_long_reads(genome, args.reads, mean_len=args.mean_len, seed=8000)
    bases = int(reads.lens.astype(np.int64).sum())
    log("[long] %d reads, %.1f Mbases in %.1fs" % (args.reads, bases / 1e6, time.time() - t1))
    for _ in range(args.warmup):
        res = ix.long_vote(reads)
    steps = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        res = ix.long_vote(reads)
        steps.append(time.perf_counter() - ts)
    sec = min(steps)
    vs, v, o = res
    log("[long] %.1f ms/step (steps %s), %d slots" % (sec * 1e3, ["%.1f" % (s * 1e3) for s in steps], len(v)))
    line = {"metric": "sublong voting step, Mbases/s (host reads -> host vote slots + location order)",
            "value": round(bases / sec / 1e6, 2), "unit": "Mbases/s",
            "reads_per_s": round(args.reads / sec, 1), "ms_per_step": round(sec * 1e3, 2),
            "steps_ms": [round(s * 1e3, 2) for s in steps], "slots": int(len(v)),
            "config": {"genome": args.genome, "index": "full one-block" if args.gap == 1 else "gapped (gap 3)",
                       "reads": args.reads, "mean_len": args.mean_len, "bases": bases,
                       "errors": "3% sub, 2% ins, 2% del"}}
    from oracle.pyoracle import OracleIndex
    oi = OracleIndex(arrays=ix.export())
    cpu = cpu_info()
    if args.check:
        sub = reads.slice(0, args.check)
        want = oi.long_vote(sub, threads=cpu["usable_cpus"])
        k = int(vs[args.check])
        same = (want[0] == vs[:args.check + 1]).all() and (want[1] == v[:k]).all() and (want[2] == o[:k]).all()
        line["parity_check"] = bool(same)
        log("[long] parity on the first %d reads: %s" % (args.check, "IDENTICAL" if same else "DIFFERENT"))
    if args.cpu_reads:
        sub = reads.slice(0, args.cpu_reads)
        sb = int(sub.lens.astype(np.int64).sum())
        ts = time.perf_counter()
        oi.long_vote(sub, threads=cpu["usable_cpus"])
        ct = time.perf_counter() - ts
        line["cpu_baseline"] = {"value": round(sb / ct / 1e6, 3), "unit": "Mbases/s", "cores": cpu["usable_cpus"],
                                "kind": "port", "sample": "first %d reads (%.1f Mbases), oracle/svoracle.c "
                                "svo_long_vote_batch, %.1f s" % (args.cpu_reads, sb / 1e6, ct),
                                "cpu_model": cpu["model"]}
        log("[long] CPU restatement %.2f Mbases/s on %d threads" % (sb / ct / 1e6, cpu["usable_cpus"]))
    print(json.dumps(line), flush=True)
    ix.close()


if __name__ == "__main__":
    main()
