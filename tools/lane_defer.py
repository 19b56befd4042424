#!/usr/bin/env python3
"""Diagnostic: share of single-end reads that leave the lane-per-read path, by reason
(candidates > CAP or read length, vote-table slots > K, shift-indel second round).
Usage: lane_defer.py [c3|c4|c5|c5pe|chr901] [n_reads]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import subread_amd as sa  # noqa: E402
from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC  # noqa: E402
from subread_amd.sim import random_genome, simulate_reads, simulate_pairs, simulate_spliced_reads, c3_lengths  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
    if wl in ("c3", "c4", "c5", "c5pe"):
        g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    else:
        g = random_genome([1_000_000], 901)
    ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True)
    if wl == "c4":
        r, r2 = simulate_pairs(g, n, 150, seed=4004)
        ix.set_max_read_length(150)
    elif wl == "c5pe":
        r, r2 = simulate_pairs(g, n, 100, seed=4004)
        ix.set_max_read_length(100)
    elif wl == "c5":
        r, r2 = simulate_spliced_reads(g, n, 100, seed=5005), None
        ix.set_max_read_length(100)
    else:
        r, r2 = simulate_reads(g, n, 100, seed=20261015, sub=0.01, indel=0.001), None
        ix.set_max_read_length(100)
    ix.set_stats(True)
    prog = PROGRAM_SUBJUNC if wl in ("c5", "c5pe") else PROGRAM_ALIGN
    ix.vote(default_params(prog, r2 is not None), r, r2)
    st, dc = ix.stats(), ix.debug_counters()
    print("%s: %d reads, %.2f hits/read, to the wave kernel %d (%.2f%%)" % (
        wl, n, st["hits"] / n, st["deferred"], 100.0 * st["deferred"] / n))
    print("  wave kernel: %d candidates settled in batch mode, %d replayed serially" % (dc[26], dc[27]))
    for name, b in (("light", 16), ("heavy", 21)):
        print("  %s pass: deferred %d (cap/length %d, slots %d, shift-indel %d), candidates voted %d" % (
            name, dc[b + 4], dc[b], dc[b + 1], dc[b + 2], dc[b + 3]))
    ix.close()


if __name__ == "__main__":
    main()
