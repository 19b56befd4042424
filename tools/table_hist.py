#!/usr/bin/env python3
"""Diagnostic (GPU box): how big the vote tables of C3 reads get, from the oracle restatement on
the bench's reads (oracle/svoracle.c svo_diag_hist): per read the most candidates one (strand,
end) table took and the most slots one table used, as a joint histogram -- what the wave kernel's
LDS table must hold.  Also the GPU lane path's deferral count on the same reads.
Usage: table_hist.py [n_reads]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, MAPPING_DTYPE  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, c3_lengths  # noqa: E402
from oracle.pyoracle import OracleIndex, lib as olib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0)
rb = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001)
p = default_params()
ix.set_stats(True)
out = np.zeros((n, 1, 3), MAPPING_DTYPE)
ix.vote(p, rb, None, bufs=(out, None, None))
st = ix.stats()
ix.set_stats(False)
oi = OracleIndex(arrays=ix.export())
L = olib()
h = (ctypes.c_uint64 * 56)()
L.svo_diag_hist(h, 1)
ref, _, _, _ = oi.vote(p, rb, None, threads=16)
L.svo_diag_hist(h, 1)
H = np.array(list(h), dtype=np.int64).reshape(7, 8)
cl = ["<=40", "41-64", "65-96", "97-128", "129-160", "161-256", ">256"]
sl = ["<=16", "<=32", "<=64", "<=128", "<=192", "<=256", "<=384", ">384"]
print("reads %d, GPU deferred %d (%.2f%%), records identical %s" % (
    n, st["deferred"], 100.0 * st["deferred"] / n, bool((ref.view(np.uint8) == out.view(np.uint8)).all())))
print("rows: most candidates in one (strand, end) table; columns: most slots used in one table")
print("%-8s" % "" + "".join("%9s" % x for x in sl) + "%10s" % "all")
for i in range(7):
    print("%-8s" % cl[i] + "".join("%9d" % x for x in H[i]) + "%10d" % H[i].sum())
print("%-8s" % "all" + "".join("%9d" % x for x in H.sum(0)) + "%10d" % H.sum())
