"""GPU box diagnostic: HIP hardware-queue sharing.  Host pipeline (packed, pinned) and the
device path on (a) a stream created after the library's copy streams, (b) the handle's own
stream.  Run with and without GPU_MAX_HW_QUEUES."""
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
dev = torch.device("cuda", 0)
p = default_params()
keep = []


def pinned(count, dt):
    dt = np.dtype(dt)
    t = torch.empty(max(1, count * dt.itemsize), dtype=torch.uint8, pin_memory=True)
    keep.append(t)
    return t.numpy()[:count * dt.itemsize].view(dt)


pk = sa.pack_reads(rb, 100, threads=16, alloc=pinned)
o = pinned(n * 3, sa.MAPPING_DTYPE).reshape(n, 1, 3)
for k in range(4):
    t = time.perf_counter()
    ix.vote_packed(p, pk, None, bufs=(o, None, None))
    print("host packed pinned %.1f Mreads/s" % (n / (time.perf_counter() - t) / 1e6), flush=True)
d = (torch.from_numpy(rb.seq).to(dev), torch.from_numpy(rb.offsets.view(np.int64)).to(dev),
     torch.from_numpy(rb.lens.view(np.int16)).to(dev))
out = torch.empty(n * 204, dtype=torch.uint8, device=dev)
ix.set_max_read_length(100)
s = torch.cuda.Stream(device=dev)
for tag, sp in (("device, new torch stream", s.cuda_stream), ("device, handle stream", None)):
    ix.vote_device(p, (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n), None, out.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        ix.vote_device(p, (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n), None, out.data_ptr(), stream=sp)
    ix.device_status()
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    print(tag, "%.1f Mreads/s" % (n * 3 / t / 1e6), flush=True)
