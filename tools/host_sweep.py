"""GPU box: host pipeline (packed reads, pinned buffers) at C3 over sub-batch sizes and
worker-thread counts, with the pipe_debug option's wait accounting."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import subread_amd as sa
from subread_amd.abi import default_params
from subread_amd.sim import random_genome, simulate_reads, c3_lengths

n = int(os.environ.get("N", 50_000_000))
g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, device=0)
rb = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001)
p = default_params()
keep = []


def pinned(count, dt):
    dt = np.dtype(dt)
    t = torch.empty(max(1, count * dt.itemsize), dtype=torch.uint8, pin_memory=True)
    keep.append(t)
    return t.numpy()[:count * dt.itemsize].view(dt)


pk = sa.pack_reads(rb, 100, threads=16, alloc=pinned)
pk.lens = pinned(n, np.uint16)
pk.lens[:] = rb.lens
o = pinned(n * 3, sa.MAPPING_DTYPE).reshape(n, 1, 3)
sa.set_option("debug", 2)
for sub in os.environ.get("SUBS", "262144 524288 1048576 2097152").split():
    for th in os.environ.get("THREADS", "8 16").split():
        sa.set_option("host_sub", int(sub))
        sa.set_option("host_threads", int(th))
        ix.vote_packed(p, pk, None, bufs=(o, None, None))
        best = 0
        for k in range(3):
            t = time.perf_counter()
            ix.vote_packed(p, pk, None, bufs=(o, None, None))
            best = max(best, n / (time.perf_counter() - t) / 1e6)
        print("sub %s threads %s: %.1f Mreads/s" % (sub, th, best), flush=True)
