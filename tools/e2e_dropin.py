#!/usr/bin/env python3
"""End to end ("report end-to-end, including the host realignment and SAM,
separately"): the reference's own subread-align run twice on the same FASTQ and index files --
stock (its CPU voting step) and the drop-in (oracle/_ref/subread-align-dropin: the same binary
with integration/do_voting_gpu.c voting on the GPU through libsubread_amd.so) -- wall time of
each whole program (index load, FASTQ parse, voting, iteration two, SAM / VCF writing), and the
outputs compared byte for byte.

Workload: a --mbp Mbp genome (contigs of GRCh38-like relative lengths, repeat families), full
one-block index files written by our builder (md5-identical to subread-buildindex -F -B),
--reads x 100 bp SE reads (1% substitutions, 0.1% indels), -T --threads.
-> one JSON line on stdout."""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mbp", type=int, default=200)
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--workdir", default="")
    ap.add_argument("--kinds", default="dump,dropin,dropin_refit2",
                    help="which binaries: dump (stock), dropin (GPU vote + the library's iteration two), "
                         "dropin_refit2 (GPU vote + the reference's own iteration two, SVG_REF_ITER2=1)")
    ap.add_argument("--out", default="", help="also write the JSON line here")
    ap.add_argument("--genome", default="synth", choices=["synth", "c3"],
                    help="synth: --mbp Mbp with repeat families; c3: bench.py's C3 genome (3.0 Gbp, 24 contigs)")
    ap.add_argument("--gpu-build", action="store_true", help="write the index files with the GPU builder "
                    "(svg_index_build_mem + save_prefix; the same bytes as the CPU builder, minutes faster at 3 Gbp)")
    ap.add_argument("--no-startup", action="store_true", help="skip the one-read runs (fixed cost) of each binary")
    ap.add_argument("--reuse", action="store_true", help="keep index files already in --workdir (the same --genome)")
    ap.add_argument("--bam", action="store_true", help="the reference's default output, BAM (no --SAMoutput)")
    ap.add_argument("--keep-order", action="store_true", help="--keepReadOrder (BAM: the ordered stream, compared byte for byte)")
    ap.add_argument("--devices", default="0,0,0,0,0,0,0,0",
                    help="SVG_DEVICES of the kind dropin_dev (default: eight replicas on device 0)")
    args = ap.parse_args()
    kinds = args.kinds.split(",")
    import subread_amd as sa
    from subread_amd.sim import c3_lengths, random_genome, simulate_reads
    from tests import dropin
    from bench import cpu_info
    cpu = cpu_info()
    T = args.threads or cpu["usable_cpus"]
    wd = args.workdir or tempfile.mkdtemp(prefix="svg_e2e_")
    os.makedirs(wd, exist_ok=True)
    t0 = time.time()
    if args.genome == "c3":   # bench.py's c3 workload genome
        g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    else:
        g = random_genome(c3_lengths(args.mbp * 1_000_000), 3000, repeats=(args.mbp * 300, 300, 200, 0.12))
    fa, pre = os.path.join(wd, "g.fa"), os.path.join(wd, "g_full")
    if args.reuse and os.path.exists(pre + ".00.b.tab") and os.path.exists(pre + ".reads"):
        log("[e2e] reusing the index files in %s" % wd)
    elif args.gpu_build:
        ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0, save_prefix=pre)
        ix.close()
    else:
        g.write_fasta(fa)
        sa.build_index(fa, pre, gap=1, force_one_block=True)
    tab_bytes = os.path.getsize(pre + ".00.b.tab")
    log("[e2e] genome %.0f Mbp + index files in %.1fs" % (g.length / 1e6, time.time() - t0))
    rb = simulate_reads(g, args.reads, 100, seed=20261015, sub=0.01, indel=0.001)
    fq, fq1 = os.path.join(wd, "r.fq"), os.path.join(wd, "r1.fq")
    dropin.write_fastq(fq, rb)
    dropin.write_fastq(fq1, rb.slice(0, 1))
    import threading
    stop = threading.Event()

    def heartbeat():   # the programs' own output is captured: keep the GPU runner's log moving
        t = time.time()
        while not stop.wait(30):
            log("[e2e] ... %.0f s" % (time.time() - t))
    threading.Thread(target=heartbeat, daemon=True).start()
    res, start, phases = {}, {}, {}
    # the reference's phase clocks on; the test harness's vote / event dumps off (tests.dropin.run turns
    # them on: ~0.6 GB written inside the before-realign window of both programs at 3M reads)
    env = {"SVG_REF_TIMING": "1", "SVG_REF_DUMP": "", "SVG_REF_EVENTS": ""}
    suffix = ".bam" if args.bam else ".sam"
    extra = ["--keepReadOrder"] if args.keep_order else []
    for kind in kinds:
        binkind = "dropin" if kind in ("dropin_refit2", "dropin_dev") else kind
        # (the drop-in's stages must all be the library's, SVG_REQUIRE_LIBRARY=1 -- but for the run that
        # asks for the reference's iteration two on purpose)
        kenv = dict(env, SVG_REF_ITER2="1", SVG_REQUIRE_LIBRARY="0") if kind == "dropin_refit2" else dict(env)
        if kind == "dropin_dev":   # the same drop-in with one replica per listed device
            kenv["SVG_DEVICES"] = args.devices
        # the fixed cost first (index load(s), voting space, output files): the same program on one read
        out = os.path.join(wd, "one_%s%s" % (kind, suffix))
        ts = time.perf_counter()
        if not args.no_startup:
            dropin.run(0, binkind, pre, fq1, None, out, threads=T, extra=extra, timeout=1500, env=kenv, sam=not args.bam)
        start[kind] = time.perf_counter() - ts
        out = os.path.join(wd, "out_%s%s" % (kind, suffix))
        ts = time.perf_counter()
        r = dropin.run(0, binkind, pre, fq, None, out, threads=T, extra=extra, timeout=1500, env=kenv, sam=not args.bam)
        res[kind] = time.perf_counter() - ts
        phases[kind] = parse_phases(r.stderr)
        log("[e2e] %s: %.1f s (%.1f s on one read) phases %s" % (kind, res[kind], start[kind], phases[kind]))
    stop.set()
    same = None
    if len(kinds) >= 2:
        for k in kinds[1:]:
            a, b = os.path.join(wd, "out_%s%s" % (kinds[0], suffix)), os.path.join(wd, "out_%s%s" % (k, suffix))
            if args.bam:
                # BAM: the records (byte for byte in order with --keepReadOrder or -T 1, else as a multiset:
                # the stock aligner's threads write their blocks unordered), and the VCF
                from tests.test_dropin import _bam_record_list, _bam_blocks_after_header
                ra, rb_ = _bam_record_list(a), _bam_record_list(b)
                if args.keep_order or T == 1:
                    assert ra == rb_ and _bam_blocks_after_header(a) == _bam_blocks_after_header(b), "BAM differs (%s)" % k
                else:
                    assert len(ra) == len(rb_) and sorted(ra) == sorted(rb_), "BAM records differ (%s)" % k
                assert open(a + ".indel.vcf", "rb").read() == open(b + ".indel.vcf", "rb").read(), "VCF differs (%s)" % k
            else:
                dropin.compare(a, b)
        same = True
        log("[e2e] %s / VCF identical (%s)" % ("BAM records" if args.bam else "SAM", ", ".join(kinds)))
    if len(kinds) == 1:
        k = kinds[0]
        line = {"metric": "end-to-end subread-align phases", "kind": k, "seconds": round(res[k], 2),
                "startup_s": round(start[k], 2), "phases": phases[k], "threads": T, "cpu_model": cpu["model"],
                "config": {"genome_mbp": round(g.length / 1e6, 1), "reads": args.reads, "read_len": 100}}
        print(json.dumps(line), flush=True)
        if args.out:
            json.dump(line, open(args.out, "w"), indent=1)
        return
    dk = kinds[1]
    res["dropin"], start["dropin"] = res[dk], start[dk]
    line = {"metric": "end-to-end subread-align (index load + parse + vote + iteration two + SAM), Mreads/s",
            "dropin_binary": "oracle/_ref/subread-align-" + dk,
            "stock_value": round(args.reads / res["dump"] / 1e6, 4), "dropin_value": round(args.reads / res["dropin"] / 1e6, 4),
            "unit": "Mreads/s", "stock_s": round(res["dump"], 2), "dropin_s": round(res["dropin"], 2),
            "speedup": round(res["dump"] / res["dropin"], 2),
            "startup_s": {"stock": round(start["dump"], 2), "dropin": round(start["dropin"], 2)},
            "mapping_only": {"stock_value": round(args.reads / max(1e-9, res["dump"] - start["dump"]) / 1e6, 4),
                             "dropin_value": round(args.reads / max(1e-9, res["dropin"] - start["dropin"]) / 1e6, 4),
                             "note": "whole-program time minus the same program's time on one read"},
            "outputs_identical": same, "threads": T,
            "dropin_refit2": ({"seconds": round(res["dropin_refit2"], 2),
                               "note": "the same drop-in with the reference's own iteration two (SVG_REF_ITER2=1)"}
                              if "dropin_refit2" in res else None),
            "dropin_dev": ({"seconds": round(res["dropin_dev"], 2), "svg_devices": args.devices,
                            "note": "the same drop-in with one index replica per SVG_DEVICES entry, each chunk's reads "
                                    "split among them (svg_index_open_devices: one read of the files)"}
                           if "dropin_dev" in res else None),
            "phases_s": phases,
            "phases_note": "the reference's own clocks (read_chunk_circles, core.c:3552-3641), printed by "
                           "oracle/ref_dump_hook.c: load_index, voting, before_realign (anti-support scan + "
                           "remove_neighbour), realign (iteration two incl. SAM writing); test dumps off",
            "cpu_model": cpu["model"],
            "config": {"genome_mbp": round(g.length / 1e6, 1), "genome": args.genome, "tab_bytes": tab_bytes,
                       "reads": args.reads, "read_len": 100, "mode": "SE, -t 1 (DNA)",
                       "output": ("BAM" if args.bam else "SAM") + (", --keepReadOrder" if args.keep_order else ""),
                       "svg_devices_of_dropin_dev": args.devices if "dropin_dev" in kinds else None,
                       "index": "full one-block files (our builder, md5-identical to subread-buildindex -F -B)"}}
    print(json.dumps(line), flush=True)
    if args.out:
        json.dump(line, open(args.out, "w"), indent=1)


def parse_phases(stderr):
    import re
    m = re.findall(r"SVG_REF_PHASES (.*)", stderr)
    if not m:
        return None
    d = {}
    for kv in m[-1].split():
        k, v = kv.split("=")
        d[k] = round(float(v), 3) if "." in v else int(v)
    # the drop-in's split of its voting phase (integration/do_voting_gpu.c)
    v = re.findall(r"SVG_DROPIN_VOTING (.*)", stderr)
    if v:
        d["voting_split"] = dict((kv.split("=")[0], round(float(kv.split("=")[1]), 3)) for kv in v[-1].split())
    st = re.findall(r"SVG_DROPIN_STAGES (.*)", stderr)
    if st:
        d["stages"] = st[-1]
    return d


if __name__ == "__main__":
    main()
