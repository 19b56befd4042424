#!/usr/bin/env python3
"""svg_probe_keys throughput (GPU box): cellCounts' prefill_votes lookups on the C3 genome's
full index (bucket-code image) and gapped index (key-hash image), keys already in HBM
(svg_probe_keys_device), image path vs the literal search (option keys_literal), and the two
paths' answers compared key for key (the literal search is the reference's procedure; the
small-index parity vs the reference itself is tests/test_gpu_prefill.py).

Keys: 16-mers at uniform random genome positions (hits) and uniform random 32-bit keys (mostly
misses), 64M each.  Prints one JSON object per (index, key set)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.sim import random_genome, c3_lengths  # noqa: E402

B2I = np.full(256, 3, np.uint32)
B2I[ord("A")], B2I[ord("G")], B2I[ord("C")] = 0, 1, 2


def genome_keys(g, n, seed):
    """genekey2int of the 16-mers at n random positions (input-files.c:1232-1251)."""
    rng = np.random.default_rng(seed)
    pos = rng.integers(0, len(g.flat) - 16, n)
    key = np.zeros(n, np.uint32)
    for i in range(16):
        key = (key << np.uint32(2)) | B2I[g.flat[pos + i]]
    return key


def run(ix, dk, n, literal, reps=5):
    dev = dk.device
    first = torch.empty(n, dtype=torch.int32, device=dev)
    count = torch.empty(n, dtype=torch.int32, device=dev)
    sa.set_option("keys_literal", 1 if literal else 0)
    L = sa.lib()

    def call():
        rc = L.svg_probe_keys_device(ix.h, 0, ctypes.c_void_p(dk.data_ptr()), n, ctypes.c_void_p(first.data_ptr()),
                                     ctypes.c_void_p(count.data_ptr()), None)
        if rc:
            raise SystemExit("svg_probe_keys_device: %s" % L.svg_last_error())
    call()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return dt, first.cpu().numpy(), count.cpu().numpy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    sets = {"genome 16-mers": genome_keys(g, n, 11), "random keys": np.random.default_rng(12).integers(0, 2 ** 32, n, dtype=np.uint32)}
    for gap, name in ((1, "C3 full index (bucket code)"), (3, "C3g gapped index (key hash)")):
        ix = sa.VoteIndex.build_genome(g, gap=gap, memory_mb=8000, force_one_block=gap == 1, device=0)
        for kname, keys in sets.items():
            dk = torch.from_numpy(keys.view(np.int32)).to("cuda:0")
            ti, fi, ci = run(ix, dk, n, False)
            tl, fl, cl = run(ix, dk, n, True)
            same = bool((ci == cl).all() and (fi[ci > 0] == fl[cl > 0]).all())
            print(json.dumps({"index": name, "keys": kname, "n_keys": n, "image_gkeys_per_s": round(n / ti / 1e9, 3),
                              "literal_gkeys_per_s": round(n / tl / 1e9, 3), "speedup": round(tl / ti, 2),
                              "hit_fraction": round(float((ci > 0).mean()), 4), "image_equals_literal": same}), flush=True)
            del dk
        ix.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
