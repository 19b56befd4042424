#!/usr/bin/env python3
"""Profiling target (GPU box): one bench workload's vote path, exactly 1 warmup + STEPS timed
steps and nothing else on the GPU, so that a rocprofv3 trace or PMC pass holds
(1 + STEPS) x launches-per-step dispatches of every vote kernel.
  MODE host   (default): the path bench.py's `value` measures -- svg_vote_batch_packed from
              2-bit packed reads in pinned host memory to records in pinned host memory
              (1M-read sub-batches: 48 launches per kernel per 50M-read step)
  MODE device: svg_vote_batch_packed_device, reads and records resident in HBM (bench.py's
              device_path figure; 6.25M-read chunks)
  name=value   library options (svg_set_option) set before the run, e.g. overlap=0 for the
              single-stream (serialised) pipeline whose kernel durations sum to at most its step
After the timed steps, host mode runs one more step with per-launch HIP events on each launch's
stream (svg_set_timing) and prints them as one JSON line ("kernel_record").
Usage: prof_run.py WORKLOAD [STEPS] [MODE] [name=value ...]   (WORKLOAD c3 | c3g | c4 | c5)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, PROGRAM_SUBJUNC, MAPPING_DTYPE, BIG_MARGIN_WORDS, SvgPackedReads  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, simulate_pairs, simulate_spliced_reads, c3_lengths  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    mode = sys.argv[3] if len(sys.argv) > 3 else "host"
    opts = dict(a.split("=", 1) for a in sys.argv[4:])
    for k, v in opts.items():
        sa.set_option(k, int(v))
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    gap = 3 if wl == "c3g" else 1
    ix = sa.VoteIndex.build_genome(g, gap=gap, memory_mb=8000, force_one_block=gap == 1, device=0)
    dev = torch.device("cuda", 0)
    if wl == "c4":
        n, L = 25_000_000, 150
        r1, r2 = simulate_pairs(g, n, L, seed=4004)
        p = default_params(paired=True)
    elif wl == "c5":
        n, L = 50_000_000, 100
        r1, r2 = simulate_spliced_reads(g, n, L, seed=5005), None
        p = default_params(PROGRAM_SUBJUNC)
    else:
        n, L = 50_000_000, 100
        r1, r2 = simulate_reads(g, n, L, seed=20261015, sub=0.01, indel=0.001), None
        p = default_params()
    keep = []
    ends = 2 if r2 is not None else 1
    sj = wl == "c5"
    if mode == "host":
        # exactly bench.py's host step: pinned packed reads (stride L), pinned records
        def pinned(count, dt):
            dt = np.dtype(dt)
            t = torch.empty(max(1, count * dt.itemsize), dtype=torch.uint8, pin_memory=True)
            keep.append(t)
            return t.numpy()[:count * dt.itemsize].view(dt)
        from subread_amd.abi import SUBJUNC_DTYPE
        pk1 = sa.pack_reads(r1, L, threads=16, alloc=pinned)
        pk2 = sa.pack_reads(r2, L, threads=16, alloc=pinned) if r2 is not None else None
        for pk, rb in ((pk1, r1), (pk2, r2)):
            if pk is not None:
                pk.lens = pinned(n, np.uint16)
                pk.lens[:] = rb.lens
        bufs = (pinned(n * ends * 3, MAPPING_DTYPE).reshape(n, ends, 3),
                pinned(n * ends * 3, SUBJUNC_DTYPE).reshape(n, ends, 3) if sj else None,
                pinned(n * ends * BIG_MARGIN_WORDS, np.uint16).reshape(n, ends, BIG_MARGIN_WORDS) if sj else None)

        def step():
            ix.vote_packed(p, pk1, pk2, bufs=bufs)
        step()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        t = time.perf_counter() - t
        print("%s host: %d reads x %d ends, %.1f ms/step, %.1f Mreads/s" % (wl, n, ends, t / steps * 1e3,
                                                                          n * ends * steps / t / 1e6))
        ix.set_timing(True)
        t1 = time.perf_counter()
        step()
        t1 = time.perf_counter() - t1
        kt = ix.kernel_timing()
        ix.set_timing(False)
        import json
        print(json.dumps({"kernel_record": {k: {"ms": round(ms, 4), "launches": nl} for k, (ms, nl) in kt.items() if nl},
                          "timed_step_ms": round(t / steps * 1e3, 3), "record_step_ms": round(t1 * 1e3, 3),
                          "workload": wl, "reads": n * ends, "options": opts}), flush=True)
        return

    def dq(rb):
        pk = sa.pack_reads(rb, L, threads=16)
        t = [torch.from_numpy(pk.bases.view(np.uint8)).to(dev), torch.from_numpy(rb.lens.view(np.uint8)).to(dev)]
        keep.append(t)
        q = SvgPackedReads()
        q.bases, q.lens, q.xmask, q.starts, q.stride, q.n_reads = t[0].data_ptr(), t[1].data_ptr(), None, None, L, n
        return q
    q1 = dq(r1)
    q2 = dq(r2) if r2 is not None else None
    out = torch.empty(n * ends * 3 * MAPPING_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    jout = torch.empty(n * ends * 3 * 16, dtype=torch.uint8, device=dev) if sj else None
    bm = torch.empty(n * ends * BIG_MARGIN_WORDS * 2, dtype=torch.uint8, device=dev) if sj else None
    ix.set_max_read_length(L)
    torch.cuda.synchronize()

    def step():
        ix.vote_packed_device(p, q1, q2, out.data_ptr(), jout.data_ptr() if sj else None, bm.data_ptr() if sj else None)
    step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    ix.device_status()
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    print("%s device: %d reads x %d ends, %.1f ms/step, %.1f Mreads/s" % (wl, n, ends, t / steps * 1e3, n * ends * steps / t / 1e6))
    # the same per-launch HIP-event record as the host mode's (one more step)
    ix.set_timing(True)
    t1 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t1
    kt = ix.kernel_timing()
    ix.set_timing(False)
    import json
    print(json.dumps({"kernel_record": {k: {"ms": round(ms, 4), "launches": nl} for k, (ms, nl) in kt.items() if nl},
                      "timed_step_ms": round(t / steps * 1e3, 3), "record_step_ms": round(t1 * 1e3, 3),
                      "workload": wl, "reads": n * ends, "mode": "device", "options": opts}), flush=True)


if __name__ == "__main__":
    main()
