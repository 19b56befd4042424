"""GPU box: device-resident C3 vote path, per-kernel times, for library variants selected by
environment switches read at launch time (A/B inside one process, same index and reads).
Usage: VARIANTS="SVG_PROBE_V1=1;" python tools/probe_ab.py  (';'-separated, ','-joined vars)"""
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
steps = int(os.environ.get("STEPS", 3))
g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, device=0)
rb = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001)
dev = torch.device("cuda", 0)
pk = sa.pack_reads(rb, 100, threads=16)
dq = [torch.from_numpy(pk.bases.view(np.uint8)).to(dev), torch.from_numpy(rb.lens.view(np.uint8)).to(dev)]
q = sa.SvgPackedReads()
q.bases, q.lens, q.xmask, q.starts, q.stride, q.n_reads = dq[0].data_ptr(), dq[1].data_ptr(), None, None, 100, n
out = torch.empty(n * 204, dtype=torch.uint8, device=dev)
p = default_params()
ix.set_max_read_length(100)
ref = None
for var in os.environ.get("VARIANTS", ";SVG_PROBE_V1=1").split(";"):
    env = dict(kv.split("=") for kv in var.split(",") if kv)
    for k, v in env.items():
        os.environ[k] = v
    ix.vote_packed_device(p, q, None, out.data_ptr())
    ix.device_status()
    torch.cuda.synchronize()
    got = out[: 2_000_000 * 204].cpu().numpy()
    same = "ref" if ref is None else ("IDENTICAL" if (got == ref).all() else "MISMATCH")
    if ref is None:
        ref = got
    ix.set_timing(True)
    t = time.perf_counter()
    for _ in range(steps):
        ix.vote_packed_device(p, q, None, out.data_ptr())
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    kt = ix.kernel_timing()
    ix.set_timing(False)
    print("%-30s %.1f Mreads/s %.1f ms/step %s" % (var or "default", n * steps / t / 1e6, t / steps * 1e3, same),
          {k: "%.2f ms x %d" % (v[0] / max(1, v[1]), v[1] // steps) for k, v in kt.items() if v[1]}, flush=True)
    for k in env:
        del os.environ[k]

ix.set_stats(True)
ix.vote_packed_device(p, q, None, out.data_ptr())
ix.device_status()
st = ix.stats()
dc = ix.debug_counters()
print("stats:", st, "big-bucket probes:", dc[5], "(%.2f%% of probes)" % (100.0 * dc[5] / max(1, st["probes"])), flush=True)
