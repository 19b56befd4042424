#!/usr/bin/env python3
"""svg_index_open of a human-sized index from files: bench.py's C3 genome (3.0 Gbp), its full
one-block index written by the GPU builder (save_prefix: the reference's .tab / .array / .reads
bytes), then opened from the files with the loader's phase clocks (option debug bit 8).
-> one JSON line (seconds per open, .tab size)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import subread_amd as sa
    from subread_amd.sim import random_genome, c3_lengths
    wd = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp(prefix="svg_open_")
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    os.makedirs(wd, exist_ok=True)
    pre = os.path.join(wd, "c3_full")
    t = time.time()
    if not os.path.exists(pre + ".00.b.tab"):
        g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
        ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0, save_prefix=pre)
        ix.close()
        del g
    print("[open] index files in %.1f s" % (time.time() - t), file=sys.stderr, flush=True)
    sa.set_option("debug", 8)
    secs = []
    for _ in range(reps):
        t = time.perf_counter()
        ix = sa.VoteIndex(pre, device=0)
        secs.append(time.perf_counter() - t)
        ix.close()
        print("[open] svg_index_open %.2f s" % secs[-1], file=sys.stderr, flush=True)
    print(json.dumps({"metric": "svg_index_open of the C3 full index files", "seconds": [round(x, 3) for x in secs],
                      "tab_bytes": os.path.getsize(pre + ".00.b.tab")}), flush=True)


if __name__ == "__main__":
    main()
