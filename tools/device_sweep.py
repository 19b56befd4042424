"""GPU box: the HBM-resident entry (svg_vote_batch_packed_device) at C3 against the host
pipeline (svg_vote_batch_packed) in one process, over device-path chunk sizes (option "chunk",
reads per chunk; 0 = the default 160 MiB of probe records), ramping and host pacing (option
dev_pace), interleaved rounds.  SETTINGS="host;chunk,ramp[,pace];..."
-> one line per setting and round (Mreads/s, ms/step)."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import subread_amd as sa
from subread_amd.abi import default_params, SvgPackedReads, MAPPING_DTYPE
from subread_amd.sim import random_genome, simulate_reads, c3_lengths

n = int(os.environ.get("N", 50_000_000))
g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, device=0)
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
o = pinned(n * 3, MAPPING_DTYPE).reshape(n, 1, 3)
dev = torch.device("cuda", 0)
tb = torch.from_numpy(pk.bases.view(np.uint8)).to(dev)
tl = torch.from_numpy(pk.lens.view(np.uint8)).to(dev)
q = SvgPackedReads()
q.bases, q.lens, q.xmask = tb.data_ptr(), tl.data_ptr(), None
q.starts, q.stride, q.n_reads = None, pk.stride, n
d_out = torch.empty(n * MAPPING_DTYPE.itemsize * 3, dtype=torch.uint8, device=dev)
ix.set_max_read_length(100)


def host():
    ix.vote_packed(p, pk, None, bufs=(o, None, None))


def device():
    ix.vote_packed_device(p, q, None, d_out.data_ptr(), None, None)


def timed(f, steps=5):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps


settings = [s.split(",") for s in os.environ.get("SETTINGS", "host;0,1;1048576,1;262144,1;0,0;1048576,0").split(";")]
for rnd in range(int(os.environ.get("ROUNDS", 2))):
    for s in settings:
        if s[0] == "host":
            dt = timed(host)
        else:
            sa.set_option("chunk", int(s[0]))
            sa.set_option("host_ramp", int(s[1]))
            sa.set_option("dev_pace", int(s[2]) if len(s) > 2 else 0)
            dt = timed(device)
            sa.set_option("chunk", 0)
            sa.set_option("host_ramp", 1)
            sa.set_option("dev_pace", 0)
        print("round %d %-16s %.1f Mreads/s %.2f ms/step" % (rnd, "/".join(s), n / dt / 1e6, dt * 1e3), flush=True)
