#!/usr/bin/env python3
"""Diagnostic (GPU box): svg_fragile_batch vs the CPU restatement on one golden case; both
window/slot arrays saved to gpurun_out/fragile_debug_<case>.npz for offline comparison."""
import os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import subread_amd as sa
from oracle.pyoracle import OracleIndex
from tests.common import Case, IndexCache

name = sys.argv[1] if len(sys.argv) > 1 else "sj_se_full_long"
c = Case(name)
d = tempfile.mkdtemp()
pre = IndexCache(d).get(c.index_key)
ix = sa.VoteIndex(pre, device=0)
gw, gs = ix.fragile(c.params, c.r1, c.r2)
cw, cs = OracleIndex(pre).fragile(c.params, c.r1, c.r2)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "fragile_debug_%s.npz" % name), gw=gw, gs=gs, cw=cw, cs=cs)
print("gpu", len(gw), len(gs), "cpu", len(cw), len(cs))
