"""CPU: the index loader's .array / .reads part (svg_host_index_load_meta, svg_host.c), which
svg_index_open runs beside the .tab's streamed upload: the packed bases of a large .array come in
8 parallel slices (pread), a small one in one fread -- either way byte for byte the file's, with
the contig table of the .reads file (gvindex_load gene-value-index.c:190-228, load_offsets
gene-algorithms.c:1293-1370)."""
import ctypes
import os

import numpy as np
import pytest

import subread_amd as sa
from tests.common import ensure_built

ensure_built()


class HostIndex(ctypes.Structure):
    _fields_ = [("nb", ctypes.c_uint32), ("items", ctypes.c_uint64), ("gap", ctypes.c_int32), ("padding", ctypes.c_int32),
                ("bstart", ctypes.c_void_p), ("keys", ctypes.c_void_p), ("vals", ctypes.c_void_p),
                ("start_point", ctypes.c_uint32), ("length", ctypes.c_uint32), ("start_base_offset", ctypes.c_uint32),
                ("values_bytes", ctypes.c_uint32), ("values", ctypes.c_void_p), ("n_chr", ctypes.c_uint32),
                ("chr_end", ctypes.c_void_p), ("chr_name", ctypes.c_void_p), ("map", ctypes.c_void_p),
                ("map_len", ctypes.c_size_t)]


@pytest.mark.parametrize("bases,start", [(200_000, 0), (50_000_003, 0), (120_000_000, 1210)])
def test_load_meta_reads_array_and_contigs(bases, start, tmp_path):
    L = sa.lib()
    rng = np.random.default_rng(bases)
    pre = str(tmp_path / "g")
    useful = (bases + start - (start - start % 4)) >> 2
    body = rng.integers(0, 256, useful + 1, dtype=np.uint8)
    with open(pre + ".00.b.array", "wb") as f:
        f.write(np.array([start, bases], np.uint32).tobytes())
        f.write(body.tobytes())
    ends = [bases // 3, 2 * bases // 3, bases]
    with open(pre + ".reads", "w") as f:
        for i, e in enumerate(ends):
            f.write("%d\tchr%d\n" % (e, i + 1))
    ix = HostIndex()
    fn = L.svg_host_index_load_meta
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(HostIndex)]
    assert fn(pre.encode(), 0, ctypes.byref(ix)) == 0
    try:
        assert (ix.start_point, ix.length, ix.values_bytes) == (start, bases, useful + 1)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * (useful + 1)).from_address(ix.values))
        assert (got == body).all()
        assert ix.n_chr == 3
        ce = np.ctypeslib.as_array((ctypes.c_uint32 * 3).from_address(ix.chr_end))
        assert list(ce) == ends
    finally:
        L.svg_host_index_free.argtypes = [ctypes.POINTER(HostIndex)]
        L.svg_host_index_free(ctypes.byref(ix))
