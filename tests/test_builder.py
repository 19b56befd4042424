"""CPU: the product index builder is byte-identical to subread-buildindex
(md5 known answers recorded from the reference, tests/golden/index_md5.json)."""
import os

import numpy as np
import pytest

import subread_amd as sa
from tests.common import ensure_built, index_md5, md5

ensure_built()


@pytest.mark.parametrize("key", sorted(index_md5()["md5"].keys()))
def test_index_md5(key, index_cache):
    index_cache.get(key)   # asserts every md5


def test_chr901_known_answers_from_reference_survey(index_cache):
    # the reference test script prints these (test/subread-align/subread-align-test.sh:8-9)
    pre = index_cache.get("chr901_full")
    assert md5(pre + ".00.b.tab") == "39cd407b95c866d7db864ce69a7d08fb"
    assert md5(pre + ".00.b.array") == "76f6c2a84c5097b13435bbeac4a8acd8"
    pre = index_cache.get("chr901_gapped")
    assert md5(pre + ".00.b.tab") == "69177bea26228055ddfa942cb26475d9"


def test_bucket_count():
    # calculate_buckets_by_size known values
    import ctypes
    L = ctypes.CDLL(sa.LIB_PATH)
    L.svg_bucket_count.restype = ctypes.c_uint32
    L.svg_bucket_count.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert L.svg_bucket_count(int(22000 * 1024 / 8) * 1024, 1) == 93018839
    assert L.svg_bucket_count(int(8000 * 1024 / 8) * 1024, 3) == 11275013


def test_builder_rejects_missing_fasta(tmp_path):
    with pytest.raises(sa.SvgError):
        sa.build_index(str(tmp_path / "nope.fa"), str(tmp_path / "x"), gap=3)


def test_builder_short_contigs_only(tmp_path):
    fa = tmp_path / "s.fa"
    fa.write_text(">a\nACGT\n>b\nACGTACGTAC\n")
    with pytest.raises(sa.SvgError):
        sa.build_index(str(fa), str(tmp_path / "x"), gap=3)
