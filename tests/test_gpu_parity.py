"""GPU parity: the HIP path (through the C ABI) reproduces the reference's vote
records byte for byte -- on the golden fixtures generated from the reference
itself, and against the oracle restatement on larger seeded read sets."""
import os

import numpy as np
import pytest

from tests.common import Case, golden_names, ensure_built, pack_records, describe_mismatch

ensure_built()
pytestmark = pytest.mark.gpu

GPU_CASES = golden_names()


@pytest.fixture(scope="module")
def gpu_indexes(index_cache):
    import subread_amd as sa
    cache = {}

    def get(key):
        if key not in cache:
            cache[key] = sa.VoteIndex(index_cache.get(key), device=0)
        return cache[key]
    yield get
    for v in cache.values():
        v.close()


@pytest.mark.parametrize("name", GPU_CASES)
def test_gpu_matches_reference_golden(name, gpu_indexes):
    c = Case(name)
    ix = gpu_indexes(c.index_key)
    out, jout, bm = ix.vote(c.params, c.r1, c.r2)
    got = pack_records(out, jout, bm)
    assert (got == c.expected).all(), describe_mismatch(got, c.expected, c.ends, c.params.multi_best)


@pytest.mark.parametrize("key,paired,n", [("chr901_full", False, 200000), ("chr901_gapped", False, 100000),
                                          ("chr901_full", True, 60000), ("synth4242_gapped", True, 40000)])
def test_gpu_matches_oracle_simulated(key, paired, n, gpu_indexes, index_cache):
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_ALIGN
    from subread_amd.sim import Genome, random_genome, simulate_reads
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    r1 = simulate_reads(g, n, 100, seed=123, sub=0.02, indel=0.02, nrate=0.002)
    r2 = simulate_reads(g, n, 100, seed=456, sub=0.02, indel=0.02) if paired else None
    p = default_params(PROGRAM_ALIGN, paired)
    out, _, _ = gpu_indexes(key).vote(p, r1, r2)
    ref, _, _, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    got = pack_records(out, None, None)
    want = pack_records(ref, None, None)
    assert (got == want).all(), describe_mismatch(got, want, 2 if paired else 1, 3)


@pytest.mark.parametrize("key,paired,n", [("chr901_full", False, 60000), ("synth4242_gapped", True, 20000),
                                          ("chr901_gapped", True, 20000)])
def test_gpu_subjunc_matches_oracle_spliced(key, paired, n, gpu_indexes, index_cache):
    """Subjunc mode (junction minor search, donor scoring, big-margin records) on
    spliced reads: ~30% of reads span a GT..AG intron of the genome."""
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_SUBJUNC
    from subread_amd.sim import Genome, simulate_spliced_reads
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    r1 = simulate_spliced_reads(g, n, 100, seed=11)
    r2 = simulate_spliced_reads(g, n, 100, seed=12) if paired else None
    p = default_params(PROGRAM_SUBJUNC, paired)
    out, jout, bm = gpu_indexes(key).vote(p, r1, r2)
    ref, rj, rbm, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    assert (rj["minor_votes"] > 0).sum() > n // 20      # the case exercises junctions
    got = pack_records(out, jout, bm)
    want = pack_records(ref, rj, rbm)
    assert (got == want).all(), describe_mismatch(got, want, 2 if paired else 1, 3)


@pytest.mark.parametrize("key,paired,length,n", [("chr901_full", False, 200, 12000), ("chr901_gapped", True, 300, 4000),
                                                 ("chr901_full", False, 600, 3000)])
def test_gpu_subjunc_long_reads_match_oracle(key, paired, length, n, gpu_indexes, index_cache):
    """Subjunc mode on reads > 160 bp (6 bp subread step, long-read junction branch with
    the halves' indel offsets; the reference's fragile junction voting only feeds event
    tables and leaves these records unchanged -- pinned by the sj_*_long goldens)."""
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_SUBJUNC
    from subread_amd.sim import Genome, simulate_spliced_reads
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    r1 = simulate_spliced_reads(g, n, length, seed=21)
    r2 = simulate_spliced_reads(g, n, length, seed=22) if paired else None
    p = default_params(PROGRAM_SUBJUNC, paired)
    out, jout, bm = gpu_indexes(key).vote(p, r1, r2)
    ref, rj, rbm, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    assert (rj["minor_votes"] > 0).sum() > n // 20
    got = pack_records(out, jout, bm)
    want = pack_records(ref, rj, rbm)
    assert (got == want).all(), describe_mismatch(got, want, 2 if paired else 1, 3)


@pytest.mark.parametrize("key,paired,length,n", [("chr901_full", False, 400, 20000), ("chr901_gapped", False, 300, 8000),
                                                 ("chr901_full", True, 250, 10000), ("chr901_full", False, 1500, 2000)])
def test_gpu_long_reads_match_oracle(key, paired, length, n, gpu_indexes, index_cache):
    """Long-read kernel variants (MAXL 1216, up to 192 subreads per strand); reads
    longer than 1209 bases are truncated like the reference's read_line."""
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_ALIGN
    from subread_amd.sim import Genome, simulate_reads, simulate_pairs
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    if paired:
        r1, r2 = simulate_pairs(g, n, length, seed=77, insert_max=900)
    else:
        r1, r2 = simulate_reads(g, n, length, seed=78, sub=0.02, indel=0.05), None
    p = default_params(PROGRAM_ALIGN, paired)
    out, _, _ = gpu_indexes(key).vote(p, r1, r2)
    ref, _, _, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    assert (out["selected_votes"][:, :, 0] > 0).mean() > 0.5
    got = pack_records(out, None, None)
    want = pack_records(ref, None, None)
    assert (got == want).all(), describe_mismatch(got, want, 2 if paired else 1, 3)


def test_gpu_batch_split_invariance(gpu_indexes, index_cache):
    """Votes are per-read independent: any batch split gives the same bytes."""
    c = Case("se_full_mixed")
    ix = gpu_indexes(c.index_key)
    whole, _, _ = ix.vote(c.params, c.r1)
    parts = [ix.vote(c.params, c.r1.slice(a, b))[0] for a, b in [(0, 1), (1, 777), (777, len(c.r1))]]
    assert (np.concatenate(parts, 0).view(np.uint8) == whole.view(np.uint8)).all()


def test_gpu_empty_batch(gpu_indexes):
    from subread_amd.abi import ReadBatch, default_params
    ix = gpu_indexes("chr901_gapped")
    out, _, _ = ix.vote(default_params(), ReadBatch.from_list([]))
    assert out.shape[0] == 0


@pytest.mark.parametrize("mode", ["se", "pe", "sj"])
def test_gpu_pipelines_match_oracle(mode, gpu_indexes, index_cache, svgopt):
    """The two pipelines: host sub-batches (option host_sub: upload / vote / download of
    neighbouring sub-batches overlap) and probe-record chunks (options chunk, overlap=1:
    the wave kernel of chunk c on a second stream beside chunk c+1's probe and lane
    kernels, double-buffered records) -- many small sub-batches and chunks, ragged tails."""
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import Genome, simulate_reads, simulate_spliced_reads
    key = "chr901_full"
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta("chr901"))
    n = 30011
    if mode == "sj":
        r1, r2 = simulate_spliced_reads(g, n, 100, seed=31), None
    else:
        r1 = simulate_reads(g, n, 100, seed=32, sub=0.02, indel=0.02)
        r2 = simulate_reads(g, n, 100, seed=33, sub=0.02, indel=0.02) if mode == "pe" else None
    p = default_params(PROGRAM_SUBJUNC if mode == "sj" else PROGRAM_ALIGN, mode == "pe")
    ref, rj, rbm, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    want = pack_records(ref, rj if mode == "sj" else None, rbm if mode == "sj" else None)
    ix = gpu_indexes(key)
    for env in ({"host_sub": 7001}, {"chunk": 2999, "overlap": 1},
                {"host_sub": 10007, "chunk": 3001, "overlap": 1}):
        for k, v in env.items():
            svgopt.set(k, v)
        out, jout, bm = ix.vote(p, r1, r2)
        for k in env:
            svgopt.reset(k)
        got = pack_records(out, jout if mode == "sj" else None, bm if mode == "sj" else None)
        assert (got == want).all(), "%s: %s" % (env, describe_mismatch(got, want, 2 if mode == "pe" else 1, 3))


def test_gpu_probe_images_match_oracle(svgopt):
    """The probe images picked at index load: 32-byte unary bucket codes (default for -F -B
    indexes), the key-hash of probe records in 32-byte sectors (no_bcode; the default of every
    index the code does not fit, e.g. gapped ones) or 64-byte lines (+ khash64), 64-byte bucket
    lines (+ no_khash), 16-bucket groups + u8 keys (+ no_bline), plain bounds + i16 keys
    (no_compact).  The genome carries repeat families, so that buckets past a code's 169 keys / a
    line's 59 keys take the big-bucket search."""
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_ALIGN
    from subread_amd.sim import random_genome, simulate_reads
    g = random_genome([3_000_000, 1_000_000], 77, repeats=(8000, 300, 10, 0.05))   # ~350 copies of many 16-mers
    r1 = simulate_reads(g, 40000, 100, seed=5, sub=0.01, indel=0.001)
    p = default_params(PROGRAM_ALIGN, False)
    want = None
    for env in ({}, {"no_bcode": 1}, {"no_bcode": 1, "khash64": 1}, {"no_bcode": 1, "no_khash": 1},
                {"no_bcode": 1, "no_khash": 1, "no_bline": 1}, {"no_compact": 1}):
        for k, v in env.items():
            svgopt.set(k, v)
        # repeat threshold 400 (-f 400): keys with up to 400 occurrences stay, so some buckets
        # exceed a code's 169 items too
        ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, repeat_threshold=400, device=0)
        for k in env:
            svgopt.reset(k)
        if want is None:
            a = ix.export()
            sizes = np.diff(a["bstart"].astype(np.int64))
            assert (sizes > 59).sum() > 200       # big buckets of the line image
            assert (sizes > 169).sum() > 0        # and of the code image
            ref, _, _, _ = OracleIndex(arrays=a).vote(p, r1, None, threads=16)
            want = pack_records(ref, None, None)
            del a
        out, _, _ = ix.vote(p, r1)
        ix.close()
        for k in env:
            svgopt.reset(k)
        got = pack_records(out, None, None)
        assert (got == want).all(), "%s: %s" % (env, describe_mismatch(got, want, 1, 3))


@pytest.mark.parametrize("key,mode,n", [("long777_fullM17", "se", 40000), ("long777_fullM17", "pe", 15000),
                                        ("long777_gappedM6", "sj", 20000), ("synth4242_fullM1", "pe", 15000)])
def test_gpu_multi_block_matches_oracle(key, mode, n, gpu_indexes, index_cache, svgopt):
    """Multi-block indexes: every block resident in HBM, voted in order, later blocks merging
    into the records the earlier ones left (core.c:3567-3613).  long777's blocks overlap by
    ~2 Mbp, so most reads are found again in several blocks.  Host pipeline with small
    sub-batches and the device entry too."""
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import Genome, simulate_reads, simulate_pairs, simulate_spliced_reads
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    if mode == "sj":
        r1, r2 = simulate_spliced_reads(g, n, 100, seed=41, max_intron=20000), None
    elif mode == "pe":
        r1, r2 = simulate_pairs(g, n, 150, seed=42)
    else:
        r1, r2 = simulate_reads(g, n, 100, seed=43, sub=0.02, indel=0.02, nrate=0.002), None
    p = default_params(PROGRAM_SUBJUNC if mode == "sj" else PROGRAM_ALIGN, mode == "pe")
    ix = gpu_indexes(key)
    assert ix.n_blocks > 1
    ref, rj, rbm, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    sj = mode == "sj"
    want = pack_records(ref, rj if sj else None, rbm if sj else None)
    ends = 2 if mode == "pe" else 1
    for env in ({}, {"host_sub": 7001}):
        for k, v in env.items():
            svgopt.set(k, v)
        out, jout, bm = ix.vote(p, r1, r2)
        for k in env:
            svgopt.reset(k)
        got = pack_records(out, jout if sj else None, bm if sj else None)
        assert (got == want).all(), "%s: %s" % (env, describe_mismatch(got, want, ends, 3))
    if not sj:
        import torch
        dev = torch.device("cuda", 0)
        keep = []

        def dr(b):
            t = [torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev) for x in (b.seq, b.offsets, b.lens)]
            keep.append(t)
            return (t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), len(b))
        d_out = torch.zeros(n * ends * p.multi_best * 68, dtype=torch.uint8, device=dev)
        ix.vote_device(p, dr(r1), dr(r2) if r2 is not None else None, d_out.data_ptr())
        ix.device_status()
        got = d_out.cpu().numpy().reshape(n, -1)
        assert (got == want).all(), "device: " + describe_mismatch(got, want, ends, 3)
