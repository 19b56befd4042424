"""Seeded synthetic genomes / reads (wrappers over svg_sim_* in libsubread_amd.so).

Workloads of BASELINE.json:
  C2  1,000,000 bp i.i.d. genome (seed 901), full one-block index, 100 bp SE reads,
      1% substitutions, 0.1% reads with one 1-5 bp indel, seed 20261015.
  C3  3.0 Gbp, 24 contigs with GRCh38-like lengths (seed 3000) + injected repeat
      families, full one-block index, 100 bp SE reads.
"""
import ctypes
import os

import numpy as np

from . import lib, ReadBatch

# GRCh38 primary chromosome lengths (chr1..22, X, Y), scaled to 3.0 Gbp for C3
GRCH38_LENGTHS = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973,
                  145138636, 138394717, 133797422, 135086622, 133275309, 114364328, 107043718,
                  101991189, 90338345, 83257441, 80373285, 58617616, 64444167, 46709983, 50818468,
                  156040895, 57227415]


class Genome:
    def __init__(self, names, seqs):
        self.names = list(names)
        self.seqs = [np.ascontiguousarray(s, dtype=np.uint8) for s in seqs]
        self.flat = np.concatenate(self.seqs) if len(self.seqs) > 1 else self.seqs[0]
        lens = np.array([len(s) for s in self.seqs], dtype=np.uint64)
        self.starts = np.zeros(len(lens), dtype=np.uint64)
        if len(lens) > 1:
            self.starts[1:] = np.cumsum(lens[:-1])
        self.lens = lens.astype(np.uint32)

    @property
    def length(self):
        return int(self.lens.astype(np.uint64).sum())

    def write_fasta(self, path, width=70):
        with open(path, "wb") as f:
            for n, s in zip(self.names, self.seqs):
                f.write(b">" + n.encode() + b"\n")
                b = s.tobytes()
                for i in range(0, len(b), width):
                    f.write(b[i:i + width] + b"\n")

    @classmethod
    def read_fasta(cls, path):
        import gzip
        op = gzip.open if str(path).endswith(".gz") else open
        names, seqs, cur = [], [], []
        with op(path, "rb") as f:
            for line in f:
                line = line.rstrip(b"\r\n")
                if not line:
                    continue
                if line[:1] == b">":
                    if names:
                        seqs.append(np.frombuffer(b"".join(cur), dtype=np.uint8))
                    names.append(line[1:].split()[0].decode())
                    cur = []
                else:
                    cur.append(line.upper())
            if names:
                seqs.append(np.frombuffer(b"".join(cur), dtype=np.uint8))
        return cls(names, seqs)


def random_genome(lengths, seed, names=None, repeats=None):
    """i.i.d. ACGT contigs; repeats = (n_copies, element_len, n_families, divergence)."""
    seqs = []
    for i, L in enumerate(lengths):
        a = np.empty(int(L), dtype=np.uint8)
        lib().svg_sim_genome(a.ctypes.data, int(L), int(seed) * 1000003 + i)
        if repeats:
            n_copies, elen, nfam, div = repeats
            share = int(n_copies * L / max(1, sum(lengths)))
            lib().svg_sim_repeats(a.ctypes.data, int(L), share, int(elen), int(nfam), float(div),
                                  int(seed) * 7 + i)
        seqs.append(a)
    if names is None:
        names = ["chr%d" % (i + 1) for i in range(len(lengths))] if len(lengths) > 1 else ["chrS%d" % seed]
    return Genome(names, seqs)


def c3_lengths(total=3_000_000_000):
    s = sum(GRCH38_LENGTHS)
    return [int(round(L * total / s)) for L in GRCH38_LENGTHS]


def simulate_reads(genome, n, length=100, seed=20261015, first=0, sub=0.01, indel=0.001, nrate=0.0,
                   threads=None, truth=False):
    """-> ReadBatch (fixed length), optionally (ReadBatch, ctg, pos, strand)."""
    seq = np.empty((n, length), dtype=np.uint8)
    tc = np.empty(n, dtype=np.uint32) if truth else None
    tp = np.empty(n, dtype=np.uint32) if truth else None
    ts = np.empty(n, dtype=np.uint8) if truth else None
    rc = lib().svg_sim_reads(genome.flat.ctypes.data, genome.starts.ctypes.data, genome.lens.ctypes.data,
                             len(genome.lens), int(first), int(n), int(length), float(sub), float(indel),
                             float(nrate), int(seed), seq.ctypes.data,
                             tc.ctypes.data if truth else None, tp.ctypes.data if truth else None,
                             ts.ctypes.data if truth else None, threads or min(16, os.cpu_count() or 1))
    if rc != 0:
        raise RuntimeError("svg_sim_reads failed %d" % rc)
    rb = ReadBatch.fixed(seq)
    return (rb, tc, tp, ts) if truth else rb


def simulate_spliced_reads(genome, n, length=100, seed=5, spliced=0.3, sub=0.005, min_intron=60,
                           max_intron=50_000):
    """RNA-seq-like reads for subjunc (config C5): a fraction `spliced` of the reads
    spans one GT..AG intron of the genome (donor 'GT' right after the first exon
    part, acceptor 'AG' right before the second), the rest are contiguous.  Exon
    part lengths are uniform in [10, length-10]; intron lengths log-uniform in
    [min_intron, max_intron] rounded up to the next AG.  Substitutions at rate
    `sub`; strand 50/50.  Deterministic in (seed, n).  -> ReadBatch."""
    rng = np.random.default_rng(seed)
    g = genome.flat
    starts = genome.starts.astype(np.int64)
    ends = starts + genome.lens.astype(np.int64)
    L = int(length)
    out = np.empty((n, L), dtype=np.uint8)
    n_sp = int(n * spliced)
    # contiguous reads
    n_ct = n - n_sp
    if n_ct:
        usable = np.maximum(genome.lens.astype(np.int64) - L - 1, 0)
        cum = np.concatenate([[0], np.cumsum(usable)])
        u = rng.integers(0, cum[-1], n_ct)
        c = np.searchsorted(cum, u, side="right") - 1
        pos = starts[c] + (u - cum[c])
        out[:n_ct] = g[pos[:, None] + np.arange(L)[None, :]]
    if n_sp:
        gt = np.flatnonzero((g[:-1] == ord("G")) & (g[1:] == ord("T"))).astype(np.int64)
        ag_end = np.flatnonzero((g[:-1] == ord("A")) & (g[1:] == ord("G"))).astype(np.int64) + 2
        got = 0
        while got < n_sp:
            m = (n_sp - got) * 2
            x = gt[rng.integers(0, len(gt), m)]                     # exon 1 ends at x (x = 'G' of GT)
            a = rng.integers(10, L - 9, m)
            d = np.exp(rng.uniform(np.log(min_intron), np.log(max_intron), m)).astype(np.int64)
            k = np.searchsorted(ag_end, x + d)
            ok = k < len(ag_end)
            y = np.where(ok, ag_end[np.minimum(k, len(ag_end) - 1)], 0)   # exon 2 starts at y
            c = np.searchsorted(ends, x, side="right")
            ok &= c < len(ends)
            cc = np.minimum(c, len(ends) - 1)
            ok &= (x - a >= starts[cc]) & (y + (L - a) <= ends[cc]) & (y - x <= max_intron * 2)
            x, a, y = x[ok], a[ok], y[ok]
            take = min(len(x), n_sp - got)
            j = np.arange(L)[None, :]
            for c0 in range(0, take, 1 << 18):
                c1 = min(take, c0 + (1 << 18))
                xa, aa, ya = x[c0:c1, None], a[c0:c1, None], y[c0:c1, None]
                out[n_ct + got + c0:n_ct + got + c1] = g[np.where(j < aa, xa - aa + j, ya + j - aa)]
            got += take
        perm = rng.permutation(n)
        out = out[perm]
    # substitutions and strand
    if sub > 0:
        alphabet = np.frombuffer(b"ACGT", dtype=np.uint8)
        for c0 in range(0, n, 1 << 20):
            blk = out[c0:c0 + (1 << 20)]
            hit = rng.random(blk.shape) < sub
            blk[hit] = alphabet[rng.integers(0, 4, int(hit.sum()))]
    rev = rng.random(n) < 0.5
    comp = np.zeros(256, dtype=np.uint8)
    comp[:] = ord("N")
    for a_, b_ in (("A", "T"), ("C", "G"), ("G", "C"), ("T", "A")):
        comp[ord(a_)] = ord(b_)
    for c0 in range(0, n, 1 << 20):
        blk, rv = out[c0:c0 + (1 << 20)], rev[c0:c0 + (1 << 20)]
        blk[rv] = comp[blk[rv][:, ::-1]]
    return ReadBatch.fixed(out)


def simulate_pairs(genome, n, length=150, seed=4004, first=0, insert_mean=300.0, insert_sd=50.0,
                   insert_max=600, sub=0.01, threads=None):
    """Paired-end reads (config C4), svg_sim_pairs: fragment length N(insert_mean,
    insert_sd) clipped to [length, insert_max], uniform start, fragment strand 50/50;
    R1 = first `length` bases of the fragment's strand, R2 = reverse complement of
    its last `length` bases (the reference's default -S fr).  Pairs
    first..first+n-1 of the stream.  -> (ReadBatch R1, ReadBatch R2)."""
    s1 = np.empty((n, length), dtype=np.uint8)
    s2 = np.empty((n, length), dtype=np.uint8)
    rc = lib().svg_sim_pairs(genome.flat.ctypes.data, genome.starts.ctypes.data, genome.lens.ctypes.data,
                             len(genome.lens), int(first), int(n), int(length), float(insert_mean),
                             float(insert_sd), int(insert_max), float(sub), int(seed), s1.ctypes.data,
                             s2.ctypes.data, threads or min(16, os.cpu_count() or 1))
    if rc != 0:
        raise RuntimeError("svg_sim_pairs failed %d" % rc)
    return ReadBatch.fixed(s1), ReadBatch.fixed(s2)


def simulate_long_reads(genome, n, mean_len=3000, seed=71, sub=0.03, ins=0.02, dele=0.02, min_len=200,
                        max_len=200_000, lengths=None):
    """Long reads (sublong): lengths log-normal around mean_len (or the given `lengths`), uniform
    start on a contig long enough, per-base substitutions / insertions / deletions at the given
    rates (ONT-like), strand 50/50.  Deterministic in (seed, n).  -> LongReads."""
    from .abi import LongReads
    rng = np.random.default_rng(seed)
    if lengths is None:
        sd = 0.6
        lengths = np.exp(rng.normal(np.log(mean_len) - sd * sd / 2, sd, n)).astype(np.int64)
        lengths = np.clip(lengths, min_len, max_len)
    lengths = np.asarray(lengths, dtype=np.int64)
    comp = np.full(256, ord("N"), dtype=np.uint8)
    for a_, b_ in (("A", "T"), ("C", "G"), ("G", "C"), ("T", "A")):
        comp[ord(a_)] = ord(b_)
    alphabet = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    for i in range(len(lengths)):
        L = int(lengths[i])
        span = int(L * (1 + dele - ins)) + 8
        ok = np.flatnonzero(genome.lens.astype(np.int64) > span + 1)
        c = int(ok[rng.integers(0, len(ok))])
        st = int(genome.starts[c]) + int(rng.integers(0, int(genome.lens[c]) - span))
        seg = genome.flat[st:st + span]
        u = rng.random(span)
        op = np.where(u < sub, 1, np.where(u < sub + ins, 2, np.where(u < sub + ins + dele, 3, 0)))
        base = np.where(op == 1, alphabet[rng.integers(0, 4, span)], seg)
        keep = op != 3
        pieces = base[keep]
        ins_at = np.flatnonzero(op[keep] == 2) + 1
        r = np.insert(pieces, ins_at, alphabet[rng.integers(0, 4, len(ins_at))])[:L]
        if rng.random() < 0.5:
            r = comp[r[::-1]]
        out.append(r.tobytes())
    return LongReads.from_list(out)


def write_fastq(path, batch, names=None):
    with open(path, "wb") as f:
        for i in range(len(batch)):
            s = batch.read(i)
            nm = names[i] if names is not None else "r%d" % i
            f.write(b"@" + nm.encode() + b"\n" + s + b"\n+\n" + b"I" * len(s) + b"\n")
