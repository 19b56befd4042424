"""Shared helpers for the parity tests: golden fixtures, index cache, record comparison."""
import glob
import gzip
import hashlib
import json
import os
import re
import subprocess

import numpy as np

from subread_amd.abi import (MAPPING_DTYPE, SUBJUNC_DTYPE, ReadBatch, SvgParams, PROGRAM_ALIGN,
                             PROGRAM_SUBJUNC)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def ensure_built():
    """Build the product library and the oracle restatement if missing (CPU-only compile)."""
    lib = os.path.join(ROOT, "subread_amd", "lib", "libsubread_amd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "subread_amd", "csrc"), "-j8"], check=True,
                       capture_output=True)
    olib = os.path.join(ROOT, "oracle", "lib", "libsvoracle.so")
    if not os.path.exists(olib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "port"], check=True, capture_output=True)


def golden_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz")))


def index_md5():
    with open(os.path.join(GOLD, "index_md5.json")) as f:
        return json.load(f)


def md5(p):
    h = hashlib.md5()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


# seeded synthetic genomes: lengths, seed (repeats 2500 copies of 300-bp elements, 16 families, 4%)
SYNTH_GENOMES = {
    "synth4242": ([300000, 250000, 17, 200000, 120000], 4242),
    # one 3 Mbp contig: a -M 17 / -M 6 build splits it deep inside (read_len > MIN_READ_SPLICING),
    # so consecutive blocks overlap by ~2 Mbp
    "long777": ([3000000, 150000, 900000], 777),
}


# sublong's vote table has 64973 rows of 51 slots: 54 copies of one element exactly 64973 bases
# apart put 54 positions of every subread of it in the same row (LRMsorted-hashtable.c:503-514)
LR_ROWS = 64973


def lrrow54_genome():
    from subread_amd.sim import Genome, random_genome
    g = random_genome([54 * LR_ROWS + 5000, 200000], 5454)
    a = g.seqs[0].copy()
    elem = random_genome([2000], 5455).seqs[0]
    for j in range(54):
        a[j * LR_ROWS + 1000:j * LR_ROWS + 3000] = elem
    return Genome(g.names, [a, g.seqs[1]])


CUSTOM_GENOMES = {"lrrow54": lrrow54_genome}


def synth_genome(gname):
    if gname in CUSTOM_GENOMES:
        return CUSTOM_GENOMES[gname]()
    from subread_amd.sim import random_genome
    lengths, seed = SYNTH_GENOMES[gname]
    return random_genome(lengths, seed, repeats=(2500, 300, 16, 0.04))


def index_recipe(key):
    """'<genome>_<mode>' -> (genome, gap, memory_mb, force_one_block).  full = -F -B -M 100,
    gapped = the defaults (-M 8000), fullM<n> / gappedM<n> = -F -M <n> / -M <n> (multi-block)."""
    gname, mode = key.rsplit("_", 1)
    if mode == "full":
        return gname, 1, 100, True
    if mode == "gapped":
        return gname, 3, 8000, False
    m = re.fullmatch(r"(full|gapped)M(\d+)", mode)
    if not m:
        raise KeyError(key)
    return gname, 1 if m.group(1) == "full" else 3, int(m.group(2)), False


def is_multi_block_key(key):
    return "M" in key.rsplit("_", 1)[1]


class IndexCache:
    """Builds the fixture indexes with OUR builder and checks them against the
    reference's md5 known answers before anything votes on them."""

    def __init__(self, root):
        self.root = root
        self.built = {}

    def genome_fasta(self, gname):
        if gname == "chr901":
            path = os.path.join(self.root, "chr901.fa")
            if not os.path.exists(path):
                with gzip.open(os.path.join(GOLD, "chr901.fa.gz"), "rb") as f, open(path, "wb") as o:
                    o.write(f.read())
            return path
        if gname in SYNTH_GENOMES or gname in CUSTOM_GENOMES:
            path = os.path.join(self.root, gname + ".fa")
            if not os.path.exists(path):
                synth_genome(gname).write_fasta(path)
            return path
        raise KeyError(gname)

    def get(self, key):
        if key in self.built:
            return self.built[key]
        import subread_amd as sa
        gname, gap, memory_mb, force = index_recipe(key)
        fa = self.genome_fasta(gname)
        pre = os.path.join(self.root, key)
        sa.build_index(fa, pre, gap=gap, memory_mb=memory_mb, force_one_block=force)
        want = index_md5()["md5"][key]
        for suf, m in want.items():
            got = md5(pre + suf)
            assert got == m, "index %s%s md5 %s != reference %s" % (key, suf, got, m)
        self.built[key] = pre
        return pre


class Case:
    def __init__(self, name):
        self.name = name
        with open(os.path.join(GOLD, name + ".json")) as f:
            self.meta = json.load(f)
        z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
        self.r1 = ReadBatch(z["r1_seq"], z["r1_off"], z["r1_len"])
        self.r2 = ReadBatch(z["r2_seq"], z["r2_off"], z["r2_len"]) if "r2_seq" in z else None
        self.expected = z["expected"]
        p = SvgParams()
        for (f, _), v in zip(p._fields_, z["params"]):
            setattr(p, f, int(v))
        self.params = p
        self.ends = 2 if self.r2 is not None else 1

    @property
    def index_key(self):
        return self.meta["index"]


def pack_records(out, jout, bm):
    n = out.shape[0]
    parts = [out.view(np.uint8).reshape(n, -1)]
    if jout is not None:
        parts.append(jout.view(np.uint8).reshape(n, -1))
    if bm is not None:
        parts.append(bm.view(np.uint8).reshape(n, -1))
    return np.concatenate(parts, 1)


def describe_mismatch(got, want, ends, mb, limit=5):
    """Human-readable first mismatches: read, end, best, field."""
    bad = np.nonzero((got != want).any(1))[0]
    lines = ["%d of %d reads differ" % (len(bad), got.shape[0])]
    names = MAPPING_DTYPE.names
    for i in bad[:limit]:
        d = np.nonzero(got[i] != want[i])[0]
        msgs = []
        for b in d[:6]:
            if b < ends * mb * 68:
                rec, off = divmod(int(b), 68)
                fld = [n for n in names if MAPPING_DTYPE.fields[n][1] <= off][-1]
                msgs.append("end%d best%d %s" % (rec // mb, rec % mb, fld))
            else:
                msgs.append("byte %d" % b)
        g = got[i, :ends * mb * 68].copy().view(MAPPING_DTYPE)
        w = want[i, :ends * mb * 68].copy().view(MAPPING_DTYPE)
        lines.append("read %d: %s\n  got  %s\n  want %s" % (i, ", ".join(msgs), g, w))
    return "\n".join(lines)
