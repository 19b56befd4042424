"""CPU: the 2-bit packed read form (svg_packed_reads, include/subread_vote.h).

svg_pack_reads (the product's host packer, threaded) must equal an independent numpy
packing -- base2int codes (subread.h:238) MSB-first in 32-bit words plus the exception
mask of characters that reverse_read complements to 'N' (input-files.c:1111) -- for
back-to-back and fixed-stride layouts, ragged and empty reads, every thread count."""
import numpy as np
import pytest

import subread_amd as sa
from subread_amd.abi import ReadBatch, PackedBatch, PACK_CODE, PACK_EXCEPTION
from tests.common import ensure_built

ensure_built()


def _reads(seed, n, maxlen, exotic):
    rng = np.random.default_rng(seed)
    alph = np.frombuffer(b"ACGTNacgtU.RYKM-*", np.uint8)
    out = []
    for _ in range(n):
        L = int(rng.integers(0, maxlen + 1))
        src = alph if rng.random() < exotic else alph[:4]
        out.append(src[rng.integers(0, len(src), L)].tobytes())
    return ReadBatch.from_list(out)


def test_base2int_table_matches_reference_macro():
    # subread.h:238  base2int(c) ((c)<'G'?((c)=='A'?0:2):((c)=='G'?1:3))
    for c in range(1, 256):
        want = (0 if c == ord("A") else 2) if c < ord("G") else (1 if c == ord("G") else 3)
        assert PACK_CODE[c] == want
    assert not PACK_EXCEPTION[[ord(x) for x in "ACGTU"]].any()
    assert PACK_EXCEPTION[[ord(x) for x in "Nacgtu.RYN-"]].all()


@pytest.mark.parametrize("stride", [None, 300, 301, 16])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_pack_reads_matches_numpy(stride, threads):
    b = _reads(7, 2500, 16 if stride == 16 else 300, 0.3)
    got = sa.pack_reads(b, stride, threads=threads)
    want = PackedBatch.pack_numpy(b, stride)
    assert (got.bases == want.bases).all()
    assert (got.xmask is None) == (want.xmask is None)
    if want.xmask is not None:
        assert (got.xmask == want.xmask).all()
    if stride is None:
        assert (got.starts == want.starts).all()


def test_pack_reads_plain_acgt_has_no_mask():
    b = _reads(8, 500, 150, 0.0)
    p = sa.pack_reads(b, 150, threads=4)
    assert p.xmask is None
    # 16 bases at a word boundary read as genekey2int's key
    r = b.read(0)
    if len(r) >= 16:
        key = 0
        for i, c in enumerate(r[:16]):
            key |= int(PACK_CODE[c]) << (30 - 2 * i)
        assert int(p.bases[0]) == key


def test_pack_reads_rejects_reads_longer_than_stride():
    b = ReadBatch.from_list([b"ACGT" * 10, b"AC"])
    with pytest.raises(sa.SvgError):
        sa.pack_reads(b, 39)


def test_pack_reads_empty():
    p = sa.pack_reads(ReadBatch.from_list([]), None)
    assert len(p) == 0
