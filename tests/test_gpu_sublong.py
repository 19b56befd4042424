"""svg_long_vote_batch (sublong's voting step on the GPU, include/subread_long.h) through the
C ABI: bit-exact against the reference's own outputs (tests/golden/sublong/sublong.npz, made by
oracle/_ref/ref-sublong: LRMdo_one_voting_read + LRMcopy_longvotes_to_itr + LRMmerge_sort,
longread-mapping.c:552-560,668-682,1317) on full and gapped indexes -- a full vote-table row,
wrapped vote counts, N / lowercase / IUPAC text, 16..64-base edge lengths -- through the image
probes, the literal go_QQ search (option keys_literal) and many small chunks
(option long_probes); against the oracle restatement on larger simulated sets."""
import os

import numpy as np
import pytest

from subread_amd.abi import LongReads
from tests.common import ensure_built
from tests.test_sublong import INDEXES, check_same, fixture

ensure_built()
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["image", "literal", "chunks"])
@pytest.mark.parametrize("key", INDEXES)
def test_gpu_sublong_matches_reference(key, mode, index_cache, svgopt):
    import subread_amd as sa
    if mode == "literal":
        svgopt.set("keys_literal", 1)
    if mode == "chunks":
        svgopt.set("long_probes", 20000)
    reads, vs, v, o = fixture(key)
    ix = sa.VoteIndex(index_cache.get(key), device=0)
    try:
        got = ix.long_vote(reads)
    finally:
        ix.close()
    check_same(got, (vs, v, o))


@pytest.mark.parametrize("key", ["chr901_full", "synth4242_gapped", "lrrow54_full"])
def test_gpu_sublong_matches_oracle_simulated(key, index_cache):
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    from subread_amd.sim import Genome, simulate_long_reads
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    reads = simulate_long_reads(g, 300, mean_len=6000, seed=sum(key.encode()))
    want = OracleIndex(pre).long_vote(reads, threads=8)
    ix = sa.VoteIndex(pre, device=0)
    try:
        got = ix.long_vote(reads)
    finally:
        ix.close()
    check_same(got, want)
    assert len(got[1]) > 10000


def test_gpu_sublong_edges(index_cache):
    import subread_amd as sa
    ix = sa.VoteIndex(index_cache.get("chr901_full"), device=0)
    try:
        vs, v, o = ix.long_vote(LongReads.from_list([]))
        assert len(vs) == 1 and len(v) == 0
        vs, v, o = ix.long_vote(LongReads.from_list([b"", b"ACGT", b"A" * 15, b"C" * 17]))
        assert list(vs) == [0, 0, 0, 0, 0]
        with pytest.raises(sa.SvgError):
            ix.long_vote(LongReads(np.zeros(1200000, np.uint8) + ord("A"), [0], [1200000]))
    finally:
        ix.close()
