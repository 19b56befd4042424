#!/usr/bin/env python3
"""Generates tests/golden/prefill/prefill.npz with the REFERENCE's own prefill_votes
(cell-counts.c:432-491, oracle/_ref/ref-prefill built from /root/reference/src by oracle/Makefile).
Runs only in the survey container (it needs /root/reference).  Per index: 2500 keys of 16-mers
taken from the genome (present, often in long repeat runs), 1500 random keys (mostly absent);
expected (bucket-local first item, run length) from the reference."""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, ROOT)
from tests.common import IndexCache  # noqa: E402
from subread_amd.sim import Genome  # noqa: E402

# (index key, block)
INDEXES = [("chr901_full", 0), ("chr901_gapped", 0), ("synth4242_full", 0), ("synth4242_gapped", 0),
           ("synth4242_fullM1", 1)]


def genome_keys(flat, n, rng):
    code = np.full(256, 3, np.uint32)
    code[ord("A")], code[ord("G")], code[ord("C")] = 0, 1, 2   # base2int, subread.h:238
    pos = rng.integers(0, len(flat) - 16, n)
    k = np.zeros(n, np.uint64)
    for i in range(16):
        k = (k << np.uint64(2)) | code[flat[pos + i]].astype(np.uint64)   # genekey2int, MSB-first
    return k.astype(np.uint32)


def main():
    ref = os.path.join(ROOT, "oracle", "_ref", "ref-prefill")
    assert os.path.exists(ref), "build oracle/_ref first (make -C oracle)"
    rng = np.random.default_rng(432)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        cache = IndexCache(d)
        for key, block in INDEXES:
            pre = cache.get(key)
            g = Genome.read_fasta(cache.genome_fasta(key.rsplit("_", 1)[0]))
            keys = np.concatenate([genome_keys(g.flat, 2500, rng), rng.integers(0, 2 ** 32, 1500, dtype=np.uint64).astype(np.uint32)])
            kf, of = os.path.join(d, "keys.u32"), os.path.join(d, "out.u32")
            keys.tofile(kf)
            subprocess.run([ref, pre, str(block), kf, of], check=True)
            r = np.fromfile(of, np.uint32).reshape(-1, 2)
            out[key + "_keys"] = keys
            out[key + "_first"] = r[:, 0].copy()
            out[key + "_count"] = r[:, 1].copy()
            out[key + "_block"] = np.array([block], np.int32)
            print(key, "present", int((r[:, 1] > 0).sum()), "max run", int(r[:, 1].max()))
    np.savez_compressed(os.path.join(HERE, "prefill.npz"), **out)


if __name__ == "__main__":
    main()
