"""CPU: the drop-in binding (integration/do_voting_gpu.c) inside the reference's own
subread-align / subjunc, with the vote answered by the CPU restatement
(oracle/dropin_oracle.c), gives the stock reference's SAM / VCF / junction BED / event table
byte for byte.  This pins the binding's host logic -- chunk reading, bigtable layout,
big-margin staging, the post-vote tail's text/quality orientation, fragile junction voting of
long subjunc reads, the multi-block run loop, -T > 1 -- apart from the kernels;
tests/test_gpu_dropin.py runs the same binding with the GPU library.  Needs the binaries
built from /root/reference (this container; skipped where they are absent)."""
import os

import pytest

from tests.common import Case, IndexCache
from tests.dropin import check_case, have


@pytest.fixture(scope="module")
def cache(tmp_path_factory):
    return IndexCache(str(tmp_path_factory.mktemp("dropin_idx")))


@pytest.mark.parametrize("name,threads", [
    ("pe_gapped_errmut", 1),            # PE align, test-err-mut pairs
    ("sj_pe_gapped_long", 1),           # subjunc PE > 160 bp: fragile junction voting in the binding
    ("sj_pe_mb_long_gappedM6", 1),      # subjunc PE on a 4-block index (block loop)
    ("sj_se_mb_synth_long_fullM1", 1),  # subjunc SE > 160 bp on a 4-block index: fragile windows per block
    ("se_gapped_mixed_n14_I16", 4),     # -n 14 -I 16, N / lowercase / IUPAC, -T 4
])
def test_oracle_dropin_matches_stock_reference(name, threads, cache, tmp_path):
    c = Case(name)
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "oracle-dropin", threads)
    assert rep["mapped"] > 0


@pytest.mark.parametrize("name,threads", [("pe_gapped_errmut", 4), ("sj_pe_gapped_long", 1)])
def test_votetime_harness_matches_stock_reference(name, threads, cache, tmp_path):
    """The CPU-baseline timing harness (oracle/ref_votetime.c: reads parsed before the clock,
    served from memory) changes nothing the aligner writes."""
    c = Case(name)
    if not have(c.meta["program"], "votetime"):
        pytest.skip("reference timing binaries not built (make -C oracle votetime)")
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "votetime", threads)
    assert rep["mapped"] > 0


def test_sublong_oracle_dropin_matches_stock(cache, tmp_path):
    """sublong with integration/lrm_voting_gpu.c as its per-read loop, votes from the restatement:
    the stock sublong's SAM byte for byte (batched fetch, vote-table rebuild, text orientation)."""
    from tests import dropin
    from tests.test_sublong import fixture
    if not os.path.exists(dropin.sublong_binary("oracle-dropin")):
        pytest.skip("oracle/_ref not built (no /root/reference)")
    reads = fixture("chr901_full")[0]
    fq = str(tmp_path / "r.fq")
    dropin.write_long_fastq(fq, reads)
    pre = cache.get("chr901_full")
    dropin.run_sublong("stock", pre, fq, str(tmp_path / "stock.sam"))
    dropin.run_sublong("oracle-dropin", pre, fq, str(tmp_path / "dropin.sam"))
    assert dropin.compare_sam(str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")) > 30
