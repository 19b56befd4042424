#!/usr/bin/env python3
"""Generates tests/golden/sublong/sublong.npz with the REFERENCE's own sublong voting step
(oracle/_ref/ref-sublong: LRMdo_one_voting_read + LRMcopy_longvotes_to_itr + LRMmerge_sort,
src/longread-one compiled in place by oracle/Makefile).  Runs only in the survey container (it
needs /root/reference).

Indexes: chr901 full / gapped, and lrrow54 full / gapped (tests/common.py: 54 copies of a
2000-base element 64973 bases apart, so a read over the element overflows one vote-table row);
the lrrow54 indexes are built by the reference's subread-buildindex and their md5 known answers
added to tests/golden/index_md5.json.  Per index: edge lengths (16..64 bases), simulated ONT-like
reads (3% substitutions, 2% insertions, 2% deletions) up to 30 kb, reads with N runs, lowercase,
IUPAC codes and U, random sequence, poly-A; on lrrow54 reads over the element and one 200 kb
error-free read (votes past 65535 wrap in the reference's unsigned short)."""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, ROOT)
from tests.common import GOLD, IndexCache, LR_ROWS, index_recipe  # noqa: E402
from subread_amd.abi import LONG_VOTE_DTYPE, LongReads  # noqa: E402
from subread_amd.sim import simulate_long_reads  # noqa: E402

INDEXES = ["chr901_full", "chr901_gapped", "lrrow54_full", "lrrow54_gapped"]
REFBIN = os.path.join(ROOT, "oracle", "_ref")


def md5(p):
    return hashlib.md5(open(p, "rb").read()).hexdigest()


def ref_md5s(cache, key, d):
    gname, gap, memory_mb, force = index_recipe(key)
    pre = os.path.join(d, "ref_" + key)
    args = [REFBIN + "/subread-buildindex", "-o", pre, "-M", str(memory_mb)]
    if gap == 1:
        args.append("-F")
    if force:
        args.append("-B")
    subprocess.run(args + [cache.genome_fasta(gname)], check=True, capture_output=True)
    return {s: md5(pre + s) for s in (".00.b.tab", ".00.b.array", ".reads")}


def edit(rng, r, kind):
    a = np.frombuffer(r, np.uint8).copy()
    L = len(a)
    if kind == "n_runs":
        for _ in range(4):
            s = int(rng.integers(0, max(1, L - 40)))
            a[s:s + int(rng.integers(1, 40))] = ord("N")
    elif kind == "lower":
        s = int(rng.integers(0, max(1, L - 300)))
        a[s:s + 300] = np.frombuffer(bytes(a[s:s + 300]).lower(), np.uint8)
    elif kind == "iupac":
        pos = rng.integers(0, L, max(1, L // 50))
        a[pos] = np.frombuffer(b"RYKMSWBDHVU.", np.uint8)[rng.integers(0, 12, len(pos))]
    return a.tobytes()


def reads_for(key, genome, rng):
    reads = []
    sim = simulate_long_reads(genome, 14, mean_len=3000, seed=int(rng.integers(1 << 30)))
    reads += [sim.read(i) for i in range(len(sim))]
    edge = simulate_long_reads(genome, 0, seed=1, lengths=[16, 17, 18, 19, 20, 21, 25, 31, 47, 64, 100, 161, 500,
                                                           1000, 12000, 30000])
    reads += [edge.read(i) for i in range(len(edge))]
    for kind in ("n_runs", "lower", "iupac"):
        reads.append(edit(rng, reads[int(rng.integers(0, 14))], kind))
    reads.append(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 3000)].tobytes())
    reads.append(b"A" * 500)
    if key.startswith("lrrow54"):
        # reads over the element (copies j * 64973 + 1000 .. + 3000 of contig 1)
        for j in (0, 7, 30, 53):
            s = j * LR_ROWS + int(rng.integers(0, 900))
            g = LongReads.from_list([genome.seqs[0][s:s + 2600].tobytes()])
            e = simulate_long_reads(type(genome)(["x"], [g.seq]), 1, seed=j + 11, lengths=[2400])
            reads.append(e.read(0))
        reads.append(genome.seqs[0][1100:2900].tobytes())                     # exact copy of the element
        reads.append(genome.seqs[0][LR_ROWS * 20:LR_ROWS * 20 + 200000].tobytes())   # 200 kb exact
    return reads


def run_ref(pre, reads, d):
    fq = os.path.join(d, "reads.fq")
    with open(fq, "wb") as f:
        for i, r in enumerate(reads):
            f.write(b"@r%d\n%s\n+\n%s\n" % (i, r, b"I" * len(r)))
    out = os.path.join(d, "out.bin")
    subprocess.run([REFBIN + "/ref-sublong", pre, fq, out], check=True)
    b = open(out, "rb").read()
    vstart, votes, order, o = [0], [], [], 0
    for _ in reads:
        n = int(np.frombuffer(b, np.uint32, 1, o)[0]); o += 4
        votes.append(np.frombuffer(b, LONG_VOTE_DTYPE, n, o)); o += 20 * n
        order.append(np.frombuffer(b, np.uint32, n, o)); o += 4 * n
        vstart.append(vstart[-1] + n)
    assert o == len(b)
    return np.array(vstart, np.uint64), np.concatenate(votes), np.concatenate(order)


def main():
    assert os.path.exists(REFBIN + "/ref-sublong"), "build oracle/_ref first (make -C oracle)"
    rng = np.random.default_rng(552)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        cache = IndexCache(d)
        mpath = os.path.join(GOLD, "index_md5.json")
        meta = json.load(open(mpath))
        for key in INDEXES:
            if key not in meta["md5"]:
                meta["md5"][key] = ref_md5s(cache, key, d)
        with open(mpath, "w") as f:
            json.dump(meta, f, indent=1)
        for key in INDEXES:
            pre = cache.get(key)
            from subread_amd.sim import Genome
            genome = Genome.read_fasta(cache.genome_fasta(key.rsplit("_", 1)[0]))
            reads = reads_for(key, genome, rng)
            lr = LongReads.from_list(reads)
            vs, v, o = run_ref(pre, reads, d)
            out[key + "_seq"], out[key + "_off"], out[key + "_len"] = lr.seq, lr.offsets, lr.lens
            out[key + "_vstart"], out[key + "_votes"], out[key + "_order"] = vs, v.view(np.uint8), o
            rows = v["slot"] >> 16
            print(key, "reads", len(reads), "slots", len(v), "max votes", int(v["votes"].max()),
                  "fullest row", int(np.bincount((rows.astype(np.int64) + (np.repeat(np.arange(len(reads)), np.diff(vs.astype(np.int64))) << 17)), minlength=1).max()))
    np.savez_compressed(os.path.join(HERE, "sublong.npz"), **out)


if __name__ == "__main__":
    main()
