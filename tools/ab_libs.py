#!/usr/bin/env python3
"""Interleaved A/B of two builds of libsubread_amd (GPU box): both libraries loaded in one
process, one index in HBM per library, bench.py's host step alternated A, B, A, B, ... so that
box-to-box and run-to-run drift hits both equally.  For compile-time knobs (make variant V=...).
Usage: ab_libs.py WORKLOAD ROUNDS LIB_A LIB_B [LIB_C ...]   (WORKLOAD c3 | c5pe); every library's
records are compared with the first's.  LIB@name=value,name=value sets library options (svg_set_option)
before each of that library's steps -- give the same build under two file names to compare options.
Compare two libraries at a time, in both orders: with five indexes in one process the first one
measured several percent off in one run (profiles/r06/r6r)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, PROGRAM_SUBJUNC, MAPPING_DTYPE, SUBJUNC_DTYPE, BIG_MARGIN_WORDS  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, simulate_pairs, c3_lengths  # noqa: E402


def main():
    wl, rounds, paths = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    if wl == "c5pe":
        n, L = 12_500_000, 100
        r1, r2 = simulate_pairs(g, n, L, seed=4004)
        p = default_params(PROGRAM_SUBJUNC, True)
    else:
        n, L = 50_000_000, 100
        r1, r2 = simulate_reads(g, n, L, seed=20261015, sub=0.01, indel=0.001), None
        p = default_params()
    sj = wl == "c5pe"
    ends = 2 if r2 is not None else 1
    keep = []

    def pinned(count, dt):
        dt = np.dtype(dt)
        t = torch.empty(max(1, count * dt.itemsize), dtype=torch.uint8, pin_memory=True)
        keep.append(t)
        return t.numpy()[:count * dt.itemsize].view(dt)
    pk1 = sa.pack_reads(r1, L, threads=16, alloc=pinned)
    pk2 = sa.pack_reads(r2, L, threads=16, alloc=pinned) if r2 is not None else None
    for pk, rb in ((pk1, r1), (pk2, r2)):
        if pk is not None:
            pk.lens = pinned(n, np.uint16)
            pk.lens[:] = rb.lens
    bufs = (pinned(n * ends * 3, MAPPING_DTYPE).reshape(n, ends, 3),
            pinned(n * ends * 3, SUBJUNC_DTYPE).reshape(n, ends, 3) if sj else None,
            pinned(n * ends * BIG_MARGIN_WORDS, np.uint16).reshape(n, ends, BIG_MARGIN_WORDS) if sj else None)
    libs, ixs, opts = [], [], []
    for k, spec in enumerate(paths):
        path, _, o = spec.partition("@")
        paths[k] = path
        opts.append([(kv.split("=")[0], int(kv.split("=")[1])) for kv in o.split(",") if kv])
        sa._lib = None
        sa.LIB_PATH = path
        libs.append(sa.lib())
        ixs.append(sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0))
    L = len(paths)
    times = [[] for _ in range(L)]
    same = [True] * L
    first = None
    def use(k):
        sa._lib = libs[k]
        for name, v in opts[k]:
            sa.set_option(name, v)

    for k in range(L):   # warm-up, and each library's records against the first's
        use(k)
        ixs[k].vote_packed(p, pk1, pk2, bufs=bufs)
        if k == 0:
            first = [b.copy() if b is not None else None for b in bufs]
        else:
            same[k] = all((x is None) or bool((x.view(np.uint8) == y.view(np.uint8)).all()) for x, y in zip(first, bufs))
    for _ in range(rounds):
        for k in range(L):
            use(k)
            t = time.perf_counter()
            ixs[k].vote_packed(p, pk1, pk2, bufs=bufs)
            times[k].append((time.perf_counter() - t) * 1e3)
    for k, path in enumerate(paths):
        t = np.array(times[k])
        path = path + ("@" + ",".join("%s=%d" % o for o in opts[k]) if opts[k] else "")
        print("%-48s median %7.1f ms/step (%s)  %.1f Mreads/s  records %s" % (os.path.basename(path), np.median(t),
              " ".join("%.1f" % x for x in t), n * ends / np.median(t) / 1e3, "identical" if same[k] else "DIFFERENT"), flush=True)


if __name__ == "__main__":
    main()
