#!/usr/bin/env python3
"""Diagnostic: per-phase share of wave cycles of the vote kernel (SVG_STAMPS build).
Run with SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so.  Shares only -- the
stamp build's run time is not a benchmark number."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, c3_lengths  # noqa: E402

sa.set_option("host_sub", 1000000000)   # one device call: the counters cover the batch


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
    if wl == "c3":
        g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    else:
        g = random_genome([1_000_000], 901)
    ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True)
    mode = sys.argv[3] if len(sys.argv) > 3 else "se"
    paired = mode in ("pe", "sjpe")
    from subread_amd.abi import PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import simulate_pairs, simulate_spliced_reads
    if mode == "pe":
        r1, r2 = simulate_pairs(g, n, 150)
        ix.set_max_read_length(150)
    elif mode == "sjpe":   # bench.py c5pe: subjunc on 100 bp pairs
        r1, r2 = simulate_pairs(g, n, 100, seed=4004)
        ix.set_max_read_length(100)
    elif mode == "sj":
        r1, r2 = simulate_spliced_reads(g, n, 100), None
        ix.set_max_read_length(100)
    else:
        r1, r2 = simulate_reads(g, n, 100, seed=20261015), None
        ix.set_max_read_length(100)
    p = default_params(PROGRAM_SUBJUNC if mode in ("sj", "sjpe") else PROGRAM_ALIGN, paired)
    ix.vote(p, r1, r2)
    ix.set_stats(True)
    t = time.time()
    ix.vote(p, r1, r2)
    dt = time.time() - t
    c = (ctypes.c_ulonglong * 32)()
    sa.lib().svg_debug_counters(ix.h, c)
    names = ["text+init", "probe", "gather", "vote(serial)", "topk", "output", "batch/junc", "bigmargin"]
    tot = sum(c[8 + k] for k in range(8))
    print("workload %s reads %d paired %s wall %.3fs probes %d items %d hits %d results %d" % (
        wl, n, paired, dt, c[0], c[1], c[2], c[3]))
    nd = c[20] if c[20] else n   # reads the wave kernel voted (lane-path deferrals)
    for k in range(8):
        print("  %-12s %6.2f%%  %8.0f cycles/read  %8.0f cycles per wave-kernel read" % (
            names[k], 100.0 * c[8 + k] / max(1, tot), c[8 + k] / n, c[8 + k] / nd))
    kt = [c[21], c[22], c[23]]   # phase K split: top-3 (acc[8]), simples after big-margin (acc[9]), pairs (acc[10])
    print("  phase K split (not in the shares above): top-3 %.0f, simples %.0f, pairs %.0f cycles per wave-kernel read"
          % tuple(x / nd for x in kt))
    print("  lane pass: defer cap/len %d, slots %d, shift %d, candidates %d, deferrals %d" % tuple(c[16:21]))
    print("  wave kernel: batch-settled %d, serially replayed %d" % (c[26], c[27]))
    print("  serial by reason: >= 2 slots in tolerance %d, one slot but spilled / d != 0 / kP1 <= last %d, "
          "exact vote whose group failed %d, opener with a neighbour or after a serial one in its row %d" % tuple(c[28:32]))


if __name__ == "__main__":
    main()
