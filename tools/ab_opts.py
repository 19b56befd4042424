#!/usr/bin/env python3
"""Interleaved A/B of library options in one process (GPU box): bench.py's C3 host step
(50M packed reads in pinned memory -> pinned records) alternated over option settings, so drift
hits every setting alike; the records of every setting are compared with the first's.
Usage: ab_opts.py ROUNDS "name=v,name=v" "name=v" ...   (an empty string = the defaults)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, MAPPING_DTYPE  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, c3_lengths  # noqa: E402


def main():
    rounds = int(sys.argv[1])
    sets = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[2:]]
    n = int(os.environ.get("N", 50_000_000))
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0)
    rb = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001)
    p = default_params()
    keep = []

    def pinned(count, dt):
        a = ix.host_alloc(count, dt)
        keep.append(a)
        return a
    pk = sa.pack_reads(rb, 100, threads=16, alloc=pinned)
    pk.lens = pinned(n, np.uint16)
    pk.lens[:] = rb.lens
    outs = [pinned(n * 3, MAPPING_DTYPE).reshape(n, 1, 3) for _ in range(2)]
    defaults = {k: sa.get_option(k) for s in sets for k in s}

    def apply(s):
        for k, v in defaults.items():
            sa.set_option(k, int(s.get(k, v)))
    times = [[] for _ in sets]
    same = [True for _ in sets]
    for k, s in enumerate(sets):   # warm-up, and each setting's records against the first's
        apply(s)
        ix.vote_packed(p, pk, None, bufs=(outs[min(k, 1)], None, None))
        if k:
            same[k] = bool((outs[1].view(np.uint8) == outs[0].view(np.uint8)).all())
    for _ in range(rounds):
        for k, s in enumerate(sets):
            apply(s)
            t = time.perf_counter()
            ix.vote_packed(p, pk, None, bufs=(outs[1], None, None))
            times[k].append((time.perf_counter() - t) * 1e3)
    for k, s in enumerate(sets):
        t = np.array(times[k])
        print("%-40s median %7.1f ms/step (%s)  %.1f Mreads/s  records %s" % (
            ",".join("%s=%s" % kv for kv in s.items()) or "(defaults)", np.median(t), " ".join("%.1f" % x for x in t),
            n / np.median(t) / 1e3, "identical" if same[k] else "DIFFERENT"), flush=True)


if __name__ == "__main__":
    main()
