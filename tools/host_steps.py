#!/usr/bin/env python3
"""Diagnostic (GPU box): per-step wall time of the packed host path at C3 (bench.py's metric
step), to see warm-up effects.  Usage: host_steps.py [steps] [reads]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, MAPPING_DTYPE  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, c3_lengths  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000_000
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, device=0)
    rb = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001)
    keep = []

    def pinned(count, dt):
        dt = np.dtype(dt)
        t = torch.empty(max(1, count * dt.itemsize), dtype=torch.uint8, pin_memory=True)
        keep.append(t)
        return t.numpy()[:count * dt.itemsize].view(dt)
    pk = sa.pack_reads(rb, 100, threads=16, alloc=pinned)
    pk.lens = pinned(n, np.uint16)
    pk.lens[:] = rb.lens
    out = pinned(n * 3, MAPPING_DTYPE).reshape(n, 1, 3)
    p = default_params()
    for s in range(steps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        ix.vote_packed(p, pk, None, bufs=(out, None, None))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print("step %2d: %.1f ms  %.1f Mreads/s" % (s, dt * 1e3, n / dt / 1e6), flush=True)


if __name__ == "__main__":
    main()
