#!/usr/bin/env python3
"""Throughput of the first post-vote stage (svg_events_*, include/subread_events.h: the tail of
do_voting's last run -- find_new_indels / find_new_junctions per record, the per-thread table merge
and the anti-supporting read scan), host C, on records of a voted batch.

The records come from the CPU restatement (test infrastructure, not timed) so that this runs on
any host; the events only read the records, the reads and the genome arrays.  Threads: the
reference keeps one event table per thread and merges them after the chunk
(finalise_indel_and_junction_thread); here T host threads each take a contiguous slice of the
reads into their own table, then one merge and one anti-support scan.
-> one JSON line on stdout."""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mbp", type=int, default=50)
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--mode", default="align", choices=["align", "subjunc"])
    args = ap.parse_args()
    import numpy as np
    import subread_amd as sa
    from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import c3_lengths, random_genome, simulate_reads, simulate_spliced_reads
    from oracle.pyoracle import OracleIndex
    from bench import cpu_info
    cpu = cpu_info()
    T = args.threads or cpu["usable_cpus"]
    wd = tempfile.mkdtemp(prefix="svg_events_")
    g = random_genome(c3_lengths(args.mbp * 1_000_000), 3000, repeats=(args.mbp * 300, 300, 200, 0.12))
    fa, pre = os.path.join(wd, "g.fa"), os.path.join(wd, "g_full")
    g.write_fasta(fa)
    sa.build_index(fa, pre, gap=1, force_one_block=True)
    sj = args.mode == "subjunc"
    rb = (simulate_spliced_reads(g, args.reads, 100, seed=5005) if sj else
          simulate_reads(g, args.reads, 100, seed=20261015, sub=0.01, indel=0.001))
    p = default_params(PROGRAM_SUBJUNC if sj else PROGRAM_ALIGN, False)
    t0 = time.time()
    out, jout, bm, _ = OracleIndex(pre).vote(p, rb, threads=cpu["usable_cpus"])
    log("[events] %d reads voted by the restatement in %.1fs" % (args.reads, time.time() - t0))
    ga = sa.GenomeArrays(pre)
    # one thread, one table
    t = sa.EventTable()
    o1 = out.copy()
    ts = time.perf_counter()
    t.add_batch(ga, p, rb, None, (o1, jout, bm))
    one = time.perf_counter() - ts
    t.close()
    # T threads, T tables, merge, anti-support
    o2 = out.copy()
    tabs = [sa.EventTable() for _ in range(T)]
    bounds = np.linspace(0, args.reads, T + 1).astype(int)

    def work(k):
        a, b = int(bounds[k]), int(bounds[k + 1])
        tabs[k].add_batch(ga, p, rb.slice(a, b), None,
                          (o2[a:b], jout[a:b] if jout is not None else None, bm[a:b] if bm is not None else None),
                          first_read=a)
    ts = time.perf_counter()
    th = [threading.Thread(target=work, args=(k,)) for k in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    t_add = time.perf_counter() - ts
    m = sa.EventTable.merge(tabs)
    t_merge = time.perf_counter() - ts - t_add
    m.anti_support(p, args.reads, 1, o2)
    t_all = time.perf_counter() - ts
    n_ev = len(m.events())
    same = bool((o1 == o2).all())
    line = {"metric": "post-vote event stage (find_new_indels / find_new_junctions + merge + anti-support), Mreads/s",
            "value": round(args.reads / t_all / 1e6, 3), "unit": "Mreads/s", "threads": T,
            "one_thread_add": round(args.reads / one / 1e6, 3),
            "seconds": {"add_batch": round(t_add, 3), "merge": round(t_merge, 3), "anti_support": round(t_all - t_add - t_merge, 3)},
            "events": n_ev, "gapped_flags_identical": same, "cpu_model": cpu["model"],
            "config": {"mode": args.mode, "genome_mbp": round(g.length / 1e6, 1), "reads": args.reads, "read_len": 100}}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
