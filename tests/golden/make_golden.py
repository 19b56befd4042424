#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE itself.

Runs only in the survey container (needs /root/reference and oracle/_ref built
by `make -C oracle ref`).  For every case it:
  1. builds the index with the reference's subread-buildindex (oracle/_ref),
     records the md5 of .tab/.array/.reads (index_md5.json),
  2. writes the reads as FASTQ and runs the reference aligner built with the
     vote-dump hook (oracle/ref_dump_hook.c) -> raw bigtable bytes per read,
  3. stores reads + expected bytes as tests/golden/<case>.npz.
Inputs are the reference's own test data (test/chr901.fa,
test/subread-align/data/test-err-mut-r{1,2}.fq.gz,
test/subjunc/data/junction-reads-{A,B}.fq) plus seeded synthetic reads made here.
The fixtures are data (inputs + expected outputs); no reference source is stored.
"""
import glob
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from subread_amd.abi import (MAPPING_DTYPE, SUBJUNC_DTYPE, EVENT_DTYPE, ReadBatch, read_fastq,  # noqa: E402
                             default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC)
from subread_amd.sim import Genome, write_fastq  # noqa: E402
from tests.common import SYNTH_GENOMES, index_recipe, synth_genome  # noqa: E402

REF = "/root/reference"
REFBIN = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.dirname(os.path.abspath(__file__))
DA = REF + "/test/subread-align/data"
DJ = REF + "/test/subjunc/data"


def md5(p):
    return hashlib.md5(open(p, "rb").read()).hexdigest()


def build_ref_index(fasta, prefix, key):
    _, gap, memory_mb, force = index_recipe(key)
    args = [REFBIN + "/subread-buildindex", "-o", prefix, "-M", str(memory_mb)]
    if gap == 1:
        args += ["-F"]
    if force:
        args += ["-B"]
    subprocess.run(args + [fasta], check=True, capture_output=True)
    files = sorted(os.path.basename(p)[len(os.path.basename(prefix)):] for p in glob.glob(prefix + ".[0-9][0-9].b.*"))
    return {s: md5(prefix + s) for s in files + [".reads"]}


def run_ref(prog, prefix, f1, f2, dump, extra=()):
    exe = REFBIN + ("/subjunc-dump" if prog == PROGRAM_SUBJUNC else "/subread-align-dump")
    if os.path.exists(dump):
        os.remove(dump)
    args = [exe, "-T", "4", "-i", prefix, "-r", f1, "-o", dump + ".sam"] + list(extra)
    if prog == PROGRAM_ALIGN:
        args += ["-t", "1"]
    if f2:
        args += ["-R", f2]
    env = dict(os.environ, SVG_REF_DUMP=dump)
    r = subprocess.run(args, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
    return np.fromfile(dump, dtype=np.uint8)


def run_ref_events(prog, prefix, f1, f2, path, extra=()):
    """The reference's event table after the voting step (-T 1: one thread table, events in
    read order) and the raw result_flags of every record (ref_dump_hook.c, SVG_REF_EVENTS)."""
    exe = REFBIN + ("/subjunc-dump" if prog == PROGRAM_SUBJUNC else "/subread-align-dump")
    if os.path.exists(path):
        os.remove(path)
    args = [exe, "-T", "1", "-i", prefix, "-r", f1, "-o", path + ".sam"] + list(extra)
    if prog == PROGRAM_ALIGN:
        args += ["-t", "1"]
    if f2:
        args += ["-R", f2]
    r = subprocess.run(args, env=dict(os.environ, SVG_REF_EVENTS=path), capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
    b = open(path, "rb").read()
    n = int(np.frombuffer(b[:8], np.uint64)[0])
    ev = np.frombuffer(b[8:8 + EVENT_DTYPE.itemsize * n], EVENT_DTYPE)
    rest = b[8 + EVENT_DTYPE.itemsize * n:]
    nr = int(np.frombuffer(rest[:8], np.uint64)[0])
    return ev, np.frombuffer(rest[8:8 + 2 * nr], np.uint16)


def save_events(name, prog, idx_prefix, r1, r2, over, tmp):
    """tests/golden/events/<case>.npz: the reference's events + raw record flags for the case's
    reads (for subjunc reads over 160 bp these include the fragile junction voting's and the
    short-exon search's events)."""
    extra = []
    if "total_subreads" in over:
        extra += ["-n", str(over["total_subreads"])]
    if "max_indel_length" in over:
        extra += ["-I", str(over["max_indel_length"])]
    f1 = os.path.join(tmp, name + "_e1.fq")
    write_fastq(f1, r1)
    f2 = None
    if r2 is not None:
        f2 = os.path.join(tmp, name + "_e2.fq")
        write_fastq(f2, r2)
    ev, flags = run_ref_events(prog, idx_prefix, f1, f2, os.path.join(tmp, name + ".ev"), extra)
    os.makedirs(os.path.join(GOLD, "events"), exist_ok=True)
    np.savez_compressed(os.path.join(GOLD, "events", name + ".npz"), events=ev.view(np.uint8).reshape(len(ev), EVENT_DTYPE.itemsize),
                        flags=flags)
    print("events", name, len(ev), "events,", int((flags & 64 > 0).sum()), "gapped records")


def take(batch, idx):
    return ReadBatch.from_list([batch.read(int(i)) for i in idx])


def mixed_reads(genome, n, seed, lengths, gapped):
    """Reads with N, lowercase runs, '.', IUPAC letters and 1-5 bp indels."""
    rng = np.random.default_rng(seed)
    g = genome.flat
    out = []
    for _ in range(n):
        L = int(rng.choice(lengths))
        s = int(rng.integers(0, len(g) - L - 10))
        r = bytearray(g[s:s + L + 5].tobytes())
        if rng.random() < 0.3:
            at = int(rng.integers(5, L - 5))
            k = int(rng.integers(1, 6))
            if rng.random() < 0.5:
                r[at:at] = bytes(rng.choice(list(b"ACGT"), k))
            else:
                del r[at:at + k]
        r = r[:L]
        for i in range(L):
            u = rng.random()
            if u < 0.01:
                r[i] = int(rng.choice(list(b"ACGT")))
            elif u < 0.013:
                r[i] = ord("N")
            elif u < 0.0135:
                r[i] = int(rng.choice(list(b".RYKMn")))
        if rng.random() < 0.05:
            a = int(rng.integers(0, L - 10))
            for i in range(a, a + 10):
                r[i] = ord(chr(r[i]).lower())
        if rng.random() < 0.5:
            comp = {65: 84, 67: 71, 71: 67, 84: 65}
            r = bytearray(comp.get(c, 78) for c in reversed(r))
        out.append(bytes(r))
    return ReadBatch.from_list(out)


def save_case(name, prog, paired, index, params_over, r1, r2, raw, ends, note):
    p = default_params(prog, paired, **params_over)
    n = len(r1)
    mb = p.multi_best
    per = ends * mb * 68 + (ends * mb * 16 if p.do_breakpoint_detection else 0) + \
        (ends * 9 * 2 if p.do_big_margin_filtering_for_junctions else 0)
    assert raw.size % per == 0, (raw.size, per)
    raw = raw.reshape(-1, per)
    assert raw.shape[0] == n, (raw.shape, n)
    arrs = dict(r1_seq=r1.seq, r1_off=r1.offsets, r1_len=r1.lens, expected=raw,
                params=np.array([getattr(p, f) for f, _ in p._fields_], dtype=np.int32))
    if r2 is not None:
        arrs.update(r2_seq=r2.seq, r2_off=r2.offsets, r2_len=r2.lens)
    np.savez_compressed(os.path.join(GOLD, name + ".npz"), **arrs)
    meta = dict(program=prog, paired=paired, index=index, params_over=params_over, n=n, note=note)
    with open(os.path.join(GOLD, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("case", name, "reads", n, "bytes/read", per)


from subread_amd.sim import simulate_spliced_reads  # noqa: E402


def main():
    tmp = tempfile.mkdtemp(prefix="svg_gold_")
    try:
        # ---- genomes and indexes
        with open(REF + "/test/chr901.fa", "rb") as f:
            fa = f.read()
        with gzip.open(os.path.join(GOLD, "chr901.fa.gz"), "wb", compresslevel=9) as f:
            f.write(fa)
        chr901 = REF + "/test/chr901.fa"
        synth = synth_genome("synth4242")
        long777 = synth_genome("long777")
        gfas = {"chr901": chr901}
        for gname, g in (("synth4242", synth), ("long777", long777)):
            gfas[gname] = os.path.join(tmp, gname + ".fa")
            g.write_fasta(gfas[gname])
        md5s = {}
        idx = {}
        keys = ["chr901_full", "chr901_gapped", "synth4242_full", "synth4242_gapped",
                # multi-block: split at contig starts (synth4242) and deep inside a 3 Mbp contig (long777)
                "synth4242_fullM1", "synth4242_gappedM1", "long777_fullM17", "long777_gappedM6"]
        for key in keys:
            pre = os.path.join(tmp, key)
            md5s[key] = build_ref_index(gfas[key.rsplit("_", 1)[0]], pre, key)
            idx[key] = pre
        recipes = {"chr901": "tests/golden/chr901.fa.gz"}
        for gname, (lengths, seed) in SYNTH_GENOMES.items():
            recipes[gname] = "subread_amd.sim.random_genome(%r, %d, repeats=(2500,300,16,0.04))" % (lengths, seed)
        with open(os.path.join(GOLD, "index_md5.json"), "w") as f:
            json.dump({"recipes": recipes,
                       "full": "gap=1 force_one_block memory_mb=100 (subread-buildindex -F -B -M 100)",
                       "gapped": "gap=3 memory_mb=8000 (subread-buildindex, defaults)",
                       "fullM<n>": "gap=1 memory_mb=n (subread-buildindex -F -M n), may be multi-block",
                       "gappedM<n>": "gap=3 memory_mb=n (subread-buildindex -M n), may be multi-block",
                       "md5": md5s}, f, indent=1)

        # ---- reference test reads
        n1, em1 = read_fastq(DA + "/test-err-mut-r1.fq.gz")
        _, em2 = read_fastq(DA + "/test-err-mut-r2.fq.gz")
        _, ja = read_fastq(DJ + "/junction-reads-A.fq")
        _, jb = read_fastq(DJ + "/junction-reads-B.fq")
        g901 = Genome.read_fasta(chr901)

        def fq(batch, tag):
            path = os.path.join(tmp, tag + ".fq")
            write_fastq(path, batch)
            return path

        cases = []
        sel = np.arange(0, 3000)
        cases.append(("se_full_errmut", PROGRAM_ALIGN, False, "chr901_full", {}, take(em1, sel), None,
                      "test-err-mut-r1 reads 0..2999"))
        sel = np.arange(3000, 6000)
        cases.append(("se_gapped_errmut", PROGRAM_ALIGN, False, "chr901_gapped", {}, take(em1, sel), None,
                      "test-err-mut-r1 reads 3000..5999"))
        sel = np.arange(6000, 8000)
        cases.append(("pe_full_errmut", PROGRAM_ALIGN, True, "chr901_full", {}, take(em1, sel), take(em2, sel),
                      "test-err-mut pairs 6000..7999"))
        sel = np.arange(8000, 10000)
        cases.append(("pe_gapped_errmut", PROGRAM_ALIGN, True, "chr901_gapped", {}, take(em1, sel), take(em2, sel),
                      "test-err-mut pairs 8000..9999"))
        sel = np.arange(0, 2000)
        cases.append(("sj_pe_gapped_junc", PROGRAM_SUBJUNC, True, "chr901_gapped", {}, take(ja, sel), take(jb, sel),
                      "junction-reads A/B pairs 0..1999"))
        sel = np.arange(2000, 4000)
        cases.append(("sj_se_full_junc", PROGRAM_SUBJUNC, False, "chr901_full", {}, take(ja, sel), None,
                      "junction-reads-A reads 2000..3999"))
        mixed = mixed_reads(g901, 2500, 11, [16, 17, 20, 36, 50, 75, 100, 101, 120, 150, 160, 161, 200, 250], False)
        cases.append(("se_full_mixed", PROGRAM_ALIGN, False, "chr901_full", {}, mixed, None,
                      "synthetic mixed reads seed 11 (N, lowercase, '.', IUPAC, indels, 16-250 bp)"))
        mixed_g = mixed_reads(g901, 2500, 12, [18, 20, 36, 50, 75, 100, 101, 120, 150, 160], True)
        cases.append(("se_gapped_mixed_n14_I16", PROGRAM_ALIGN, False, "chr901_gapped",
                      {"total_subreads": 14, "max_indel_length": 16}, mixed_g, None,
                      "synthetic mixed reads seed 12, -n 14 -I 16"))
        sr1, sr2 = [], []
        rng = np.random.default_rng(99)
        for i in range(2000):
            c = int(rng.integers(0, len(synth.seqs)))
            s = synth.seqs[c]
            if len(s) < 1000:
                c = 0
                s = synth.seqs[0]
            L = int(rng.choice([75, 100, 150]))
            ins = int(rng.integers(L, 600))
            st = int(rng.integers(0, len(s) - ins - 1))
            a = s[st:st + L].tobytes()
            b = s[st + ins - L:st + ins].tobytes()
            comp = {65: 84, 67: 71, 71: 67, 84: 65}
            b = bytes(comp.get(x, 78) for x in reversed(b))
            if rng.random() < 0.5:
                a, b = b, a
            sr1.append(a)
            sr2.append(b)
        cases.append(("pe_full_synth", PROGRAM_ALIGN, True, "synth4242_full", {}, ReadBatch.from_list(sr1),
                      ReadBatch.from_list(sr2), "synthetic multi-contig repeat genome seed 4242, pairs seed 99"))
        cases.append(("se_gapped_synth", PROGRAM_ALIGN, False, "synth4242_gapped", {}, ReadBatch.from_list(sr1), None,
                      "synthetic multi-contig repeat genome seed 4242, R1 of pairs seed 99"))
        # long reads (161..1210 bp: 6 bp subread step, up to 63 subreads x gap per strand)
        cases.append(("se_full_long", PROGRAM_ALIGN, False, "chr901_full", {},
                      mixed_reads(g901, 600, 13, [161, 255, 256, 257, 300, 500, 800, 1000, 1210], False), None,
                      "synthetic mixed long reads seed 13 (161-1210 bp)"))
        cases.append(("se_gapped_long", PROGRAM_ALIGN, False, "chr901_gapped", {},
                      mixed_reads(g901, 400, 14, [170, 200, 400, 700, 1210], True), None,
                      "synthetic mixed long reads seed 14 (170-1210 bp, up to 189 subreads per strand)"))
        lr1, lr2 = [], []
        rng = np.random.default_rng(15)
        g = g901.flat
        for i in range(400):
            L = int(rng.choice([200, 250, 400]))
            ins = int(rng.integers(L, 700))
            st = int(rng.integers(0, len(g) - ins - 1))
            a = g[st:st + L].tobytes()
            comp = {65: 84, 67: 71, 71: 67, 84: 65}
            b = bytes(comp.get(x, 78) for x in reversed(g[st + ins - L:st + ins].tobytes()))
            if rng.random() < 0.5:
                a, b = b, a
            lr1.append(a)
            lr2.append(b)
        cases.append(("pe_full_long", PROGRAM_ALIGN, True, "chr901_full", {}, ReadBatch.from_list(lr1),
                      ReadBatch.from_list(lr2), "chr901 pairs seed 15, 200/250/400 bp, fragments up to 700 bp"))
        # subjunc long reads (161-400 bp: 6 bp subread step; the junction search adds the indel
        # offsets of both halves); ~30% span a GT..AG intron of chr901
        sj_long = [simulate_spliced_reads(g901, 200, L, seed=16 + L) for L in (170, 250, 400)]
        sj_long = ReadBatch.from_list([b.read(i) for b in sj_long for i in range(len(b))])
        cases.append(("sj_se_full_long", PROGRAM_SUBJUNC, False, "chr901_full", {}, sj_long, None,
                      "chr901 spliced reads 170/250/400 bp, seeds 186/266/416"))
        sj_l1 = [simulate_spliced_reads(g901, 150, L, seed=30 + L) for L in (200, 300)]
        sj_l2 = [simulate_spliced_reads(g901, 150, L, seed=40 + L) for L in (200, 300)]
        cases.append(("sj_pe_gapped_long", PROGRAM_SUBJUNC, True, "chr901_gapped", {},
                      ReadBatch.from_list([b.read(i) for b in sj_l1 for i in range(len(b))]),
                      ReadBatch.from_list([b.read(i) for b in sj_l2 for i in range(len(b))]),
                      "chr901 spliced read pairs 200/300 bp, seeds 230/330 and 240/340"))
        # ---- multi-block indexes (blocks voted in order, later blocks merge with the stored records)
        cases.append(("se_mb_synth_fullM1", PROGRAM_ALIGN, False, "synth4242_fullM1", {},
                      mixed_reads(synth, 2500, 21, [50, 75, 100, 120, 150, 200], False), None,
                      "synth4242 mixed reads seed 21 on the 4-block -F -M 1 index"))
        cases.append(("pe_mb_synth_gappedM1", PROGRAM_ALIGN, True, "synth4242_gappedM1", {}, ReadBatch.from_list(sr1),
                      ReadBatch.from_list(sr2), "synth4242 pairs seed 99 on the 2-block -M 1 index"))
        cases.append(("sj_se_mb_synth_fullM1", PROGRAM_SUBJUNC, False, "synth4242_fullM1", {},
                      simulate_spliced_reads(synth, 2000, 100, seed=22, max_intron=20000), None,
                      "synth4242 spliced reads seed 22 (100 bp) on the 4-block -F -M 1 index"))
        from subread_amd.sim import simulate_pairs
        lp1, lp2 = simulate_pairs(long777, 2000, 150, seed=23, sub=0.01)
        cases.append(("pe_mb_long_fullM17", PROGRAM_ALIGN, True, "long777_fullM17", {}, lp1, lp2,
                      "long777 pairs seed 23 (150 bp) on the 6-block -F -M 17 index (blocks overlap ~2 Mbp)"))
        cases.append(("se_mb_long_gappedM6", PROGRAM_ALIGN, False, "long777_gappedM6", {},
                      mixed_reads(long777, 2500, 24, [36, 75, 100, 150, 250], True), None,
                      "long777 mixed reads seed 24 on the 4-block -M 6 index"))
        sj_lp1 = simulate_spliced_reads(long777, 1500, 150, seed=25, max_intron=20000)
        sj_lp2 = simulate_spliced_reads(long777, 1500, 150, seed=26, max_intron=20000)
        cases.append(("sj_pe_mb_long_gappedM6", PROGRAM_SUBJUNC, True, "long777_gappedM6", {}, sj_lp1, sj_lp2,
                      "long777 spliced reads seeds 25/26 (150 bp) on the 4-block -M 6 index"))
        # subjunc long reads on a 4-block index: fragile junction voting in every block's run
        sj_mbl = [simulate_spliced_reads(synth, 300, L, seed=27 + L, max_intron=20000) for L in (200, 300)]
        cases.append(("sj_se_mb_synth_long_fullM1", PROGRAM_SUBJUNC, False, "synth4242_fullM1", {},
                      ReadBatch.from_list([b.read(i) for b in sj_mbl for i in range(len(b))]), None,
                      "synth4242 spliced reads 200/300 bp, seeds 227/327, on the 4-block -F -M 1 index"))
        only = set(a for a in sys.argv[1:] if not a.startswith("--"))
        if only:
            cases = [c for c in cases if c[0] in only]
        if "--events-only" in sys.argv:
            # event tables for the committed cases (reads from their fixtures)
            from tests.common import Case
            for name, prog, paired, ikey, over, r1, r2, note in cases:
                cs = Case(name)
                save_events(name, prog, idx[ikey], cs.r1, cs.r2, over, tmp)
            return

        for name, prog, paired, ikey, over, r1, r2, note in cases:
            extra = []
            if "total_subreads" in over:
                extra += ["-n", str(over["total_subreads"])]
            if "max_indel_length" in over:
                extra += ["-I", str(over["max_indel_length"])]
            f1 = fq(r1, name + "_1")
            f2 = fq(r2, name + "_2") if r2 is not None else None
            raw = run_ref(prog, idx[ikey], f1, f2, os.path.join(tmp, name + ".bin"), extra)
            save_case(name, prog, paired, ikey, over, r1, r2, raw, 2 if paired else 1, note)
            save_events(name, prog, idx[ikey], r1, r2, over, tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
