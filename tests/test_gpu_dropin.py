"""GPU: the reference's own subread-align / subjunc with integration/do_voting_gpu.c as its
voting step (votes by libsubread_amd.so on the GPU) gives the stock reference's outputs byte
for byte: SAM (iteration two and the SAM writer of the reference consume the GPU records),
.indel.vcf, .junction.bed, plus the vote records and the event table after the voting step
(oracle/ref_dump_hook.c in both binaries).  Cases: the golden fixtures' reads (test-err-mut
PE, junction-reads A/B, long subjunc reads with fragile junction voting, -n 14 -I 16, multi-block
indexes, -T 4) and 200k C2 reads (1 Mbp seed-901 genome, full one-block index)."""
import os

import numpy as np
import pytest

from tests.common import Case, IndexCache
from tests.dropin import assert_library, case_extra, check_case, compare, fastq_pair, have, run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cache(tmp_path_factory):
    return IndexCache(str(tmp_path_factory.mktemp("gpu_dropin_idx")))


def _need(program):
    if not have(program, "dropin"):
        pytest.fail("oracle/_ref drop-in binaries missing: build them in the survey container (make -C oracle dropin)")


@pytest.mark.parametrize("name,threads", [
    ("pe_gapped_errmut", 1),            # PE align, test-err-mut pairs 8000..9999
    ("pe_full_errmut", 1),              # PE align, full index
    ("sj_pe_gapped_junc", 1),           # subjunc PE, junction-reads A/B
    ("sj_se_full_junc", 1),             # subjunc SE, big-margin records, full index
    ("sj_pe_gapped_long", 1),           # subjunc PE > 160 bp (fragile junction voting, GPU windows)
    ("sj_se_full_long", 1),             # subjunc SE 170-400 bp
    ("se_gapped_mixed_n14_I16", 4),     # -n 14 -I 16, N / lowercase / IUPAC, -T 4
    ("se_mb_synth_fullM1", 1),          # 4-block full index
    ("pe_mb_synth_gappedM1", 1),        # 2-block gapped index
    ("sj_pe_mb_long_gappedM6", 1),      # subjunc PE, 4-block index, blocks overlapping ~2 Mbp
    ("sj_se_mb_synth_long_fullM1", 1),  # subjunc SE > 160 bp, 4-block index: GPU fragile windows per block
])
def test_gpu_dropin_matches_stock_reference(name, threads, cache, tmp_path):
    c = Case(name)
    _need(c.meta["program"])
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "dropin", threads)
    assert rep["mapped"] > 0
    print(name, rep)


@pytest.mark.parametrize("name,threads", [
    ("pe_gapped_errmut", 1), ("sj_pe_gapped_junc", 1), ("sj_pe_mb_long_gappedM6", 1), ("se_gapped_mixed_n14_I16", 4)])
def test_gpu_dropin_two_handles(name, threads, cache, tmp_path):
    """SVG_DEVICES=0,0: two handles (two index replicas; this box has one GPU, so both on device 0),
    each chunk split into two contiguous read ranges voted by two host threads into the one
    bigtable -- the stock outputs byte for byte.  On an 8-GPU node SVG_DEVICES=0,...,7 gives each
    device one range."""
    c = Case(name)
    _need(c.meta["program"])
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "dropin", threads, env={"SVG_DEVICES": "0,0"})
    assert rep["mapped"] > 0


@pytest.mark.parametrize("name,threads,chunk", [("pe_gapped_errmut", 4, 600), ("sj_pe_gapped_long", 1, 0)])
def test_gpu_dropin_bam_keep_read_order(name, threads, chunk, cache, tmp_path):
    """BAM output with --keepReadOrder through the GPU drop-in (library iteration two, BAM sink):
    the record blocks after the header are byte-identical to the stock aligner's, here also across
    read chunks (SVG_REF_READS_PER_CHUNK in both programs)."""
    from tests.test_dropin import _bam_blocks_after_header, _bam_record_list
    c = Case(name)
    _need(c.meta["program"])
    f1, f2 = fastq_pair(str(tmp_path), c.name, c.r1, c.r2)
    pre = cache.get(c.index_key)
    env = {"SVG_REF_READS_PER_CHUNK": str(chunk)} if chunk else None
    so, do = str(tmp_path / "stock.bam"), str(tmp_path / "dropin.bam")
    extra = case_extra(c) + ["--keepReadOrder"]
    run(c.meta["program"], "dump", pre, f1, f2, so, threads, extra, env=env, sam=False)
    assert_library(run(c.meta["program"], "dropin", pre, f1, f2, do, threads, extra, env=env, sam=False).stderr)
    assert _bam_record_list(so) == _bam_record_list(do)
    assert _bam_blocks_after_header(so) == _bam_blocks_after_header(do)


@pytest.mark.timeout(600)
def test_gpu_dropin_c2_200k(tmp_path):
    """200k C2 reads (bench.py workload c2's genome and read generator) through the drop-in, -T 8."""
    _need(0)
    import subread_amd as sa
    from subread_amd.sim import random_genome, simulate_reads
    g = random_genome([1_000_000], 901)
    fa = str(tmp_path / "c2.fa")
    g.write_fasta(fa)
    pre = str(tmp_path / "c2_full")
    sa.build_index(fa, pre, gap=1, force_one_block=True)
    rb = simulate_reads(g, 200_000, 100, seed=20261015, first=0, sub=0.01, indel=0.001)
    f1, _ = fastq_pair(str(tmp_path), "c2", rb, None)
    so, do = str(tmp_path / "c2.stock.sam"), str(tmp_path / "c2.dropin.sam")
    run(0, "dump", pre, f1, None, so, threads=8)
    assert_library(run(0, "dropin", pre, f1, None, do, threads=8).stderr)
    rep = compare(so, do)
    # the same with two handles (contiguous halves of the chunk)
    do2 = str(tmp_path / "c2.dropin2.sam")
    assert_library(run(0, "dropin", pre, f1, None, do2, threads=8, env={"SVG_DEVICES": "0,0"}).stderr)
    compare(so, do2)
    # the reference's default output, BAM, unordered at -T 8: the same records
    from tests.test_dropin import _bam_record_list
    sb, db = str(tmp_path / "c2.stock.bam"), str(tmp_path / "c2.dropin.bam")
    run(0, "dump", pre, f1, None, sb, threads=8, sam=False)
    assert_library(run(0, "dropin", pre, f1, None, db, threads=8, sam=False).stderr)
    a, b = _bam_record_list(sb), _bam_record_list(db)
    assert len(a) == 200_000 and sorted(a) == sorted(b)
    votes = np.fromfile(do + ".votes", dtype=np.uint8)
    assert votes.size == 200_000 * 3 * 68
    assert rep["sam_records"] >= 200_000 and rep["mapped"] > 190_000, rep
    print("c2", rep)


@pytest.mark.parametrize("key,n_sim,threads", [
    ("chr901_full", 150, 1),     # the sublong fixture's reads (edges, N / lowercase / IUPAC) + simulated ONT-like reads
    ("lrrow54_full", 60, 1),     # reads over 54 element copies (a full vote-table row) and a 200 kb read
    ("chr901_full", 150, 4),     # -T 4: threads share the GPU handle
])
def test_gpu_sublong_dropin_matches_stock(key, n_sim, threads, cache, tmp_path):
    """The reference's own sublong with integration/lrm_voting_gpu.c as its per-read loop (votes
    by svg_long_vote_batch on the GPU): the stock sublong's SAM byte for byte -- the reference's
    LRMdo_dynamic_programming_read (copy, location sort, windows, chains, gap filling, SAM)
    consumes the GPU vote tables."""
    from subread_amd.abi import LongReads
    from subread_amd.sim import Genome, simulate_long_reads
    from tests import dropin
    from tests.test_sublong import fixture
    if not os.path.exists(dropin.sublong_binary("dropin")):
        pytest.fail("oracle/_ref sublong binaries missing: build them in the survey container (make -C oracle)")
    fx = fixture(key)[0]
    g = Genome.read_fasta(cache.genome_fasta(key.rsplit("_", 1)[0]))
    sim = simulate_long_reads(g, n_sim, mean_len=4000, seed=77)
    reads = LongReads.from_list([fx.read(i) for i in range(len(fx))] + [sim.read(i) for i in range(len(sim))])
    fq = str(tmp_path / "r.fq")
    dropin.write_long_fastq(fq, reads)
    pre = cache.get(key)
    dropin.run_sublong("stock", pre, fq, str(tmp_path / "stock.sam"), threads=threads)
    dropin.run_sublong("dropin", pre, fq, str(tmp_path / "dropin.sam"), threads=threads)
    assert dropin.compare_sam(str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam"), any_order=threads > 1) > n_sim
