#!/usr/bin/env python3
"""The full-size C2 digest (SURVEY.md §8(c) fixture plan), produced by the REFERENCE itself.

Runs only in the survey container (needs /root/reference and `make -C oracle ref`):
  1. the C2 genome (bench.py workload c2: 1,000,000 bp i.i.d., seed 901) written as FASTA and
     indexed by the reference's own subread-buildindex -F -B (md5 checked against our builder's);
  2. the 10M C2 reads (simulate_reads(seed 20261015, sub 0.01, indel 0.001), 100 bp) as FASTQ;
  3. the reference aligner with the vote-dump hook (oracle/_ref/subread-align-dump, -T 8) dumps
     every read's 3 mapping_result_t (68 B each, CORE_IS_GAPPED_READ cleared -- the records at
     the vote boundary) in read order;
  4. tests/golden/c2_digest.json: SHA-256 of that dump (the canonical little-endian records,
     n x 3 x 68 bytes), of each 1M-read block, and the record statistics.
tests/test_gpu_digest.py votes the same reads through svg_vote_batch_packed and compares.
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

REFBIN = os.path.join(ROOT, "oracle", "_ref")
N = 10_000_000
BLOCK = 1_000_000


def md5(p):
    h = hashlib.md5()
    with open(p, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def main():
    import subread_amd as sa
    from subread_amd.sim import random_genome, simulate_reads
    tmp = tempfile.mkdtemp(prefix="svg_c2_", dir=os.environ.get("SVG_TMP", "/tmp"))
    try:
        t0 = time.time()
        g = random_genome([1_000_000], 901)
        fa = os.path.join(tmp, "c2.fa")
        g.write_fasta(fa)
        ref_pre, our_pre = os.path.join(tmp, "c2_ref"), os.path.join(tmp, "c2_ours")
        subprocess.run([REFBIN + "/subread-buildindex", "-F", "-B", "-o", ref_pre, fa], check=True, capture_output=True)
        sa.build_index(fa, our_pre, gap=1, force_one_block=True)
        for suf in (".00.b.tab", ".00.b.array", ".reads"):
            assert md5(ref_pre + suf) == md5(our_pre + suf), suf
        print("index built and md5-checked in %.1fs" % (time.time() - t0), flush=True)
        rb = simulate_reads(g, N, 100, seed=20261015, first=0, sub=0.01, indel=0.001)
        fq = os.path.join(tmp, "c2.fq")
        seq = rb.seq.reshape(N, 100)
        with open(fq, "wb") as f:
            q = b"I" * 100
            for a in range(0, N, 100_000):
                b = min(N, a + 100_000)
                f.write(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, seq[i].tobytes(), q) for i in range(a, b)))
        print("reads written in %.1fs" % (time.time() - t0), flush=True)
        dump = os.path.join(tmp, "c2.votes")
        r = subprocess.run([REFBIN + "/subread-align-dump", "-T", "8", "-t", "1", "-i", ref_pre, "-r", fq,
                            "-o", os.path.join(tmp, "c2.bam")], env=dict(os.environ, SVG_REF_DUMP=dump),
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        print("reference run in %.1fs" % (time.time() - t0), flush=True)
        raw = np.fromfile(dump, dtype=np.uint8)
        assert raw.size == N * 3 * 68, raw.size
        rec = raw.reshape(N, 3 * 68)
        blocks = [hashlib.sha256(rec[a:a + BLOCK].tobytes()).hexdigest() for a in range(0, N, BLOCK)]
        from subread_amd.abi import MAPPING_DTYPE
        m = raw.view(MAPPING_DTYPE).reshape(N, 3)
        out = {
            "workload": "C2 (bench.py c2): random_genome([1000000], 901); simulate_reads(n=10000000, length=100, "
                        "seed=20261015, first=0, sub=0.01, indel=0.001); subread-align defaults (SE, -t 1)",
            "index": "subread-buildindex -F -B (md5-identical to svg_build_index)",
            "producer": "oracle/_ref/subread-align-dump -T 8 (the reference aligner built from /root/reference/src, "
                        "oracle/ref_dump_hook.c), records at the vote boundary",
            "records": "n x 3 x 68 B mapping_result_t, read order, little-endian, CORE_IS_GAPPED_READ cleared",
            "n_reads": N,
            "sha256": hashlib.sha256(raw.tobytes()).hexdigest(),
            "block_reads": BLOCK,
            "block_sha256": blocks,
            "reads_with_votes": int((m["selected_votes"][:, 0] > 0).sum()),
            "records_with_votes": int((m["selected_votes"] > 0).sum()),
        }
        json.dump(out, open(os.path.join(ROOT, "tests", "golden", "c2_digest.json"), "w"), indent=1)
        print(json.dumps({k: out[k] for k in ("sha256", "reads_with_votes", "records_with_votes")}))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
