"""sublong's voting step (LRMdo_one_voting_read + LRMcopy_longvotes_to_itr + LRMmerge_sort,
src/longread-one/longread-mapping.c:552-560,668-682,1317): the oracle restatement
(oracle/svoracle.c svo_long_vote_batch) against the reference's own outputs
(tests/golden/sublong/sublong.npz, made by oracle/_ref/ref-sublong from the reference source)
on full and gapped indexes, incl. a genome whose element copies overflow a 51-slot vote-table
row and a 200 kb read whose vote count wraps; the GPU entry (svg_long_vote_batch) is tested
against the same vectors in test_gpu_sublong.py."""
import os

import numpy as np
import pytest

from subread_amd.abi import LONG_VOTE_DTYPE, LongReads
from tests.common import GOLD, ensure_built

ensure_built()
FIX = os.path.join(GOLD, "sublong", "sublong.npz")
INDEXES = ["chr901_full", "chr901_gapped", "lrrow54_full", "lrrow54_gapped"]


def fixture(key):
    z = np.load(FIX, allow_pickle=False)
    reads = LongReads(z[key + "_seq"], z[key + "_off"], z[key + "_len"])
    return reads, z[key + "_vstart"], z[key + "_votes"].view(LONG_VOTE_DTYPE), z[key + "_order"]


def check_same(got, want):
    vs, v, o = got
    wvs, wv, wo = want
    assert (vs == wvs).all(), "per-read slot counts differ: first read %d" % int(np.flatnonzero(vs != wvs)[0])
    bad = np.flatnonzero(v != wv)
    assert len(bad) == 0, "slot %d differs: got %s want %s" % (bad[0], v[bad[0]], wv[bad[0]])
    bad = np.flatnonzero(o != wo)
    assert len(bad) == 0, "sort order differs at %d" % bad[0]


@pytest.mark.parametrize("key", INDEXES)
def test_oracle_sublong_matches_reference(key, index_cache):
    from oracle.pyoracle import OracleIndex
    reads, vs, v, o = fixture(key)
    got = OracleIndex(index_cache.get(key)).long_vote(reads, threads=4)
    check_same(got, (vs, v, o))
    rows = v["slot"] >> 16
    assert len(v) > 1000 and (o != np.arange(len(o), dtype=np.uint32)).any()
    if key.startswith("lrrow54"):
        assert ((v["slot"] & 0xffff) == 50).any()    # a row filled to its 51 slots
        assert rows.max() < 64973


def test_long_reads_struct_roundtrip():
    r = LongReads.from_list([b"ACGT" * 10, b"", b"N" * 5])
    assert len(r) == 3 and r.read(0) == b"ACGT" * 10 and r.read(1) == b"" and r.read(2) == b"NNNNN"
    s = r.struct()
    assert s.n_reads == 3
