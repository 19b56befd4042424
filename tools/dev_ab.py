"""GPU box diagnostic: device-resident vote path (svg_vote_batch_device) at C3, per-kernel
times, before and after a host-pipeline run.  SVG_LIB selects the library build."""
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
steps = int(os.environ.get("STEPS", 5))
g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, device=0)
rb = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001)
dev = torch.device("cuda", 0)
d = (torch.from_numpy(rb.seq).to(dev), torch.from_numpy(rb.offsets.view(np.int64)).to(dev),
     torch.from_numpy(rb.lens.view(np.int16)).to(dev))
out = torch.empty(n * 204, dtype=torch.uint8, device=dev)
p = default_params()
ix.set_max_read_length(100)
s = torch.cuda.Stream(device=dev)


def run(tag):
    ix.vote_device(p, (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n), None, out.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    ix.set_timing(True)
    t = time.perf_counter()
    for _ in range(steps):
        ix.vote_device(p, (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n), None, out.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    kt = ix.kernel_timing()
    ix.set_timing(False)
    print(tag, "%.1f Mreads/s %.1f ms/step" % (n * steps / t / 1e6, t / steps * 1e3),
          {k: "%.2f ms x %d" % (v[0] / max(1, v[1]), v[1] // steps) for k, v in kt.items() if v[1]}, flush=True)


run("device")
if hasattr(sa.lib(), "svg_vote_batch_packed") and os.environ.get("HOST", "1") == "1":
    pk = sa.pack_reads(rb, 100, threads=16)
    o = np.empty((n, 1, 3), sa.MAPPING_DTYPE)
    t = time.perf_counter()
    ix.vote_packed(p, pk, None, bufs=(o, None, None))
    print("host packed (pageable out) %.1f Mreads/s" % (n / (time.perf_counter() - t) / 1e6), flush=True)
    run("device-after-host")
