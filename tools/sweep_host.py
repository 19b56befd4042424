#!/usr/bin/env python3
"""Option sweep on the host path (GPU box): one index build, then for each configuration (library
options, svg_set_option) 1 warmup + STEPS timed steps of bench.py's host step.
Usage: sweep_host.py WORKLOAD STEPS 'NAME:opt=V,opt=V' ...   (an empty config list = baseline only)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, PROGRAM_SUBJUNC, MAPPING_DTYPE, SUBJUNC_DTYPE, BIG_MARGIN_WORDS  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, simulate_pairs, simulate_spliced_reads, c3_lengths  # noqa: E402


def main():
    wl, steps = sys.argv[1], int(sys.argv[2])
    confs = [("baseline", {})]
    for a in sys.argv[3:]:
        name, _, kv = a.partition(":")
        confs.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    gap = 3 if wl == "c3g" else 1
    ix = sa.VoteIndex.build_genome(g, gap=gap, memory_mb=8000, force_one_block=gap == 1, device=0)
    sj = wl in ("c5", "c5pe")
    if wl == "c4":
        n, L = 25_000_000, 150
        r1, r2 = simulate_pairs(g, n, L, seed=4004)
        p = default_params(paired=True)
    elif wl == "c5":
        n, L = 50_000_000, 100
        r1, r2 = simulate_spliced_reads(g, n, L, seed=5005), None
        p = default_params(PROGRAM_SUBJUNC)
    elif wl == "c5pe":
        n, L = 12_500_000, 100
        r1 = simulate_spliced_reads(g, n, L, seed=5005)
        r2 = simulate_spliced_reads(g, n, L, seed=5006)
        p = default_params(PROGRAM_SUBJUNC, True)
    else:
        n, L = 50_000_000, 100
        r1, r2 = simulate_reads(g, n, L, seed=20261015, sub=0.01, indel=0.001), None
        p = default_params()
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
    for name, env in confs:
        old = {k: sa.get_option(k) for k in env}
        for k, v in env.items():
            sa.set_option(k, int(v))
        ix.vote_packed(p, pk1, pk2, bufs=bufs)
        t = time.perf_counter()
        for _ in range(steps):
            ix.vote_packed(p, pk1, pk2, bufs=bufs)
        t = time.perf_counter() - t
        print("%-12s %-40s %7.1f ms/step %7.1f Mreads/s" % (name, ",".join("%s=%s" % kv for kv in env.items()),
                                                             t / steps * 1e3, n * ends * steps / t / 1e6), flush=True)
        for k, v in old.items():
            sa.set_option(k, v)


if __name__ == "__main__":
    main()
