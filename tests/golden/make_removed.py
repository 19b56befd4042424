#!/usr/bin/env python3
"""Generate tests/golden/events_rn/<case>.npz from the REFERENCE itself: the event types after
remove_neighbour (core-indel.c:447, run by read_chunk_circles right after the anti-supporting
read scan, core.c:3629-3630; a removed event has type 0).

Runs only in the survey container (needs oracle/_ref's subread-align-dump / subjunc-dump,
built with oracle/ref_dump_hook.c, whose SVG_REF_EVENTS_RN dump follows remove_neighbour).
For every case of tests/golden/events/ it runs the reference on the case's reads and index
exactly as make_golden.py's save_events does (-T 1, the same FASTQ), checks that the event
table it dumps before remove_neighbour is the committed one byte for byte (same inputs), and
stores the types after it.  Fixture = data (one byte per event); no reference source is stored.
"""
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.common import Case, IndexCache  # noqa: E402
from tests.golden.make_golden import run_ref_events, write_fastq  # noqa: E402
from tests.test_events import EVENT_CASES, load_events  # noqa: E402

GOLD = os.path.dirname(os.path.abspath(__file__))


def synthetic(tmp, cache):
    """Two data sets on which remove_neighbour removes events (the golden cases remove none):
    rn_se -- subread-align, 300k 100-bp reads with 2% indels over a 150 kb genome (same-length
    indels within 3 bases of each other); rn_sj -- subjunc, 30k RNA-seq reads (half spliced,
    introns up to 3 kb) over a 1.7 Mbp genome with repeat families (junctions within 11 bases).
    Stored: the reference's event table before remove_neighbour and the types after it."""
    from subread_amd import build_index
    from subread_amd.abi import PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import random_genome, simulate_reads, simulate_spliced_reads
    sets = [("rn_se", PROGRAM_ALIGN, ([150_000], 78, None), lambda g: simulate_reads(g, 300000, 100, seed=4, sub=0.005, indel=0.02)),
            ("rn_sj", PROGRAM_SUBJUNC, ([1_000_000, 700_000], 77, (200, 300, 20, 0.02)),
             lambda g: simulate_spliced_reads(g, 30000, 100, seed=6, spliced=0.5, max_intron=3000))]
    for name, prog, (lengths, seed, rep), make_reads in sets:
        g = random_genome(lengths, seed, repeats=rep)
        fa, pre = os.path.join(tmp, name + ".fa"), os.path.join(tmp, name + "_idx")
        g.write_fasta(fa)
        build_index(fa, pre, gap=1, force_one_block=True)
        f1 = os.path.join(tmp, name + ".fq")
        write_fastq(f1, make_reads(g))
        rn = os.path.join(tmp, name + ".rn")
        os.environ["SVG_REF_EVENTS_RN"] = rn
        ev, _ = run_ref_events(prog, pre, f1, None, os.path.join(tmp, name + ".ev"))
        del os.environ["SVG_REF_EVENTS_RN"]
        b = open(rn, "rb").read()
        n = int(np.frombuffer(b[:8], np.uint64)[0])
        assert n == len(ev) and len(b) == 8 + n, name
        types = np.frombuffer(b[8:], np.uint8).copy()
        np.savez_compressed(os.path.join(GOLD, "events_rn", name + ".npz"), types=types,
                            events=ev.view(np.uint8).reshape(len(ev), -1))
        print("events_rn", name, n, "events,", int((types == 0).sum()), "removed")


def main():
    tmp = tempfile.mkdtemp(prefix="svg_rn_")
    cache = IndexCache(tmp)
    os.makedirs(os.path.join(GOLD, "events_rn"), exist_ok=True)
    try:
        for name in EVENT_CASES:
            c = Case(name)
            over = c.meta["params_over"]
            extra = []
            if "total_subreads" in over:
                extra += ["-n", str(over["total_subreads"])]
            if "max_indel_length" in over:
                extra += ["-I", str(over["max_indel_length"])]
            f1 = os.path.join(tmp, name + "_e1.fq")
            write_fastq(f1, c.r1)
            f2 = None
            if c.r2 is not None:
                f2 = os.path.join(tmp, name + "_e2.fq")
                write_fastq(f2, c.r2)
            rn = os.path.join(tmp, name + ".rn")
            if os.path.exists(rn):
                os.remove(rn)
            os.environ["SVG_REF_EVENTS_RN"] = rn
            ev, _ = run_ref_events(c.meta["program"], cache.get(c.index_key), f1, f2, os.path.join(tmp, name + ".ev"), extra)
            del os.environ["SVG_REF_EVENTS_RN"]
            want, _ = load_events(name)
            assert len(ev) == len(want) and (ev.view(np.uint8) == want.view(np.uint8).reshape(-1)).all(), name
            b = open(rn, "rb").read()
            n = int(np.frombuffer(b[:8], np.uint64)[0])
            assert n == len(ev) and len(b) == 8 + n, name
            types = np.frombuffer(b[8:], np.uint8).copy()
            np.savez_compressed(os.path.join(GOLD, "events_rn", name + ".npz"), types=types)
            print("events_rn", name, n, "events,", int((types == 0).sum()), "removed")
        synthetic(tmp, cache)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
