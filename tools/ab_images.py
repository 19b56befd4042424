#!/usr/bin/env python3
"""Interleaved A/B of index-load options (probe images) on one GPU, in one process.

Every configuration gets its own index in HBM (options are read when the index is built), the
same 2-bit packed reads and pinned output are shared, and the host steps (and optionally the
HBM-resident entry's steps) alternate between the configurations round after round, so box drift
and thermal state fall on all of them alike.  Prints one JSON object: per configuration the
median / min ms per step and the per-launch kernel times of one extra step.

    python tools/ab_images.py --config base: --config kinline:kinline=1 \
        --config khash:khash_probe=1 --rounds 8 --out gpurun_out/ab.json
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--reads", type=int, default=0)
    ap.add_argument("--config", action="append", default=[],
                    help="name:opt=v,opt=v (options applied while this configuration's index is built)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--device", action="store_true", help="also alternate the HBM-resident entry")
    ap.add_argument("--hipmalloc", action="store_true",
                    help="HBM-resident entry: records into a hipMalloc'd array instead of a torch tensor")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch
    import bench
    import subread_amd as sa
    from subread_amd.abi import default_params, PROGRAM_ALIGN, MAPPING_DTYPE, SvgPackedReads
    from subread_amd.sim import random_genome, simulate_reads

    W = bench.workload(args.workload)
    if W["kind"] != "se":
        raise SystemExit("ab_images: single-end workloads only")
    n = args.reads or W["reads"]
    L = W["read_len"]
    genome = random_genome(W["lengths"], W["gseed"], repeats=W["repeats"])
    configs = []
    for c in args.config or ["base:"]:
        name, _, opts = c.partition(":")
        kv = [o.split("=", 1) for o in opts.split(",") if o]
        prev = [(k, sa.get_option(k)) for k, _ in kv]
        for k, v in kv:
            sa.set_option(k, int(v))
        t0 = time.time()
        ix = sa.VoteIndex.build_genome(genome, gap=W.get("gap", 1), memory_mb=8000, force_one_block=True, device=0)
        for k, v in prev:   # back to what it was (options read at index load only)
            sa.set_option(k, v)
        print("[ab] %s: index %.1f GB in %.1fs" % (name, ix.info.device_bytes / 1e9, time.time() - t0),
              file=sys.stderr, flush=True)
        configs.append({"name": name, "opts": dict((k, int(v)) for k, v in kv), "ix": ix, "ms": [], "dev_ms": []})

    keep = []
    ix0 = configs[0]["ix"]

    def pinned(count, dt):
        a = ix0.host_alloc(count, dt)
        keep.append(a)
        return a
    rb = simulate_reads(genome, n, L, seed=20261015, first=0, sub=0.01, indel=0.001)
    pk = sa.pack_reads(rb, L, threads=16, alloc=pinned)
    pk.lens = pinned(n, np.uint16)
    pk.lens[:] = rb.lens
    p = default_params(PROGRAM_ALIGN, False)
    out = pinned(n * p.multi_best, MAPPING_DTYPE).reshape(n, 1, p.multi_best)
    dev = torch.device("cuda", 0)
    if args.device:
        tb = torch.from_numpy(pk.bases.view(np.uint8)).to(dev)
        tl = torch.from_numpy(pk.lens.view(np.uint8)).to(dev)
        q = SvgPackedReads()
        q.bases, q.lens, q.xmask, q.starts, q.stride, q.n_reads = tb.data_ptr(), tl.data_ptr(), None, None, pk.stride, n
        if args.hipmalloc:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            ptr = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(n * MAPPING_DTYPE.itemsize * p.multi_best)) == 0

            class _Raw:
                def data_ptr(self):
                    return ptr.value
            d_out = _Raw()
        else:
            d_out = torch.empty(n * MAPPING_DTYPE.itemsize * p.multi_best, dtype=torch.uint8, device=dev)
        for c in configs:
            c["ix"].set_max_read_length(L)

    ref = None
    for c in configs:   # warm-up + an output comparison between the configurations
        c["ix"].vote_packed(p, pk, None, bufs=(out, None, None))
        sample = out[::37].copy()   # every 37th read's records
        c["identical_to_first"] = ref is None or bool(np.array_equal(sample.view(np.uint8), ref.view(np.uint8)))
        ref = sample if ref is None else ref
    for r in range(args.rounds):
        for c in (configs if r % 2 == 0 else configs[::-1]):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c["ix"].vote_packed(p, pk, None, bufs=(out, None, None))
            torch.cuda.synchronize()
            c["ms"].append((time.perf_counter() - t0) * 1e3)
            if args.device:
                t0 = time.perf_counter()
                c["ix"].vote_packed_device(p, q, None, d_out.data_ptr(), None, None)
                torch.cuda.synchronize()
                c["dev_ms"].append((time.perf_counter() - t0) * 1e3)
        print("[ab] round %d: %s" % (r, ", ".join("%s %.1f" % (c["name"], c["ms"][-1]) for c in configs)),
              file=sys.stderr, flush=True)
    res = {"workload": args.workload, "reads": n, "rounds": args.rounds, "configs": []}
    for c in configs:
        c["ix"].set_timing(True)
        c["ix"].vote_packed(p, pk, None, bufs=(out, None, None))
        kt = c["ix"].kernel_timing()
        c["ix"].set_timing(False)
        e = {"name": c["name"], "opts": c["opts"], "device_gb": round(c["ix"].info.device_bytes / 1e9, 2),
             "ms_median": round(statistics.median(c["ms"]), 2), "ms_min": round(min(c["ms"]), 2),
             "mreads_s": round(n / statistics.median(c["ms"]) / 1e3, 1),
             "identical_to_first": c["identical_to_first"], "kernels": kt}
        if c["dev_ms"]:
            e["dev_ms_median"] = round(statistics.median(c["dev_ms"]), 2)
            e["dev_mreads_s"] = round(n / statistics.median(c["dev_ms"]) / 1e3, 1)
            c["ix"].set_timing(True)
            c["ix"].vote_packed_device(p, q, None, d_out.data_ptr(), None, None)
            torch.cuda.synchronize()
            e["dev_kernels"] = c["ix"].kernel_timing()
            c["ix"].set_timing(False)
        res["configs"].append(e)
    s = json.dumps(res, indent=1)
    print(s)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
