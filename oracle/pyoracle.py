"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU restatement (oracle/svoracle.c).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg -- as the checker, never as the thing measured or shipped.
"""
import ctypes
import os
import subprocess

import numpy as np

from subread_amd.abi import MAPPING_DTYPE, SUBJUNC_DTYPE, BIG_MARGIN_WORDS

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libsvoracle.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build(quiet=True):
    """Compile the restatement (and, when /root/reference exists, oracle/_ref)."""
    out = subprocess.run(["make", "-C", HERE, "-j8"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.svo_index_open.restype = ctypes.c_void_p
        L.svo_index_open.argtypes = [ctypes.c_char_p]
        L.svo_index_close.argtypes = [ctypes.c_void_p]
        L.svo_index_info.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 5
        L.svo_prefill.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_void_p]
        L.svo_index_from_arrays.restype = ctypes.c_void_p
        L.svo_index_from_arrays.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.svo_vote_batch.restype = ctypes.c_int
        L.svo_vote_batch.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int, ctypes.c_void_p]
        L.svo_fragile_batch.restype = ctypes.c_int
        L.svo_fragile_batch.argtypes = [ctypes.c_void_p] * 5
        L.svo_fragile_free.argtypes = [ctypes.c_void_p]
        L.svo_long_vote_batch.restype = ctypes.c_int
        L.svo_long_vote_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.svo_long_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


class OracleIndex:
    def __init__(self, prefix=None, arrays=None):
        self._keep = None
        if arrays is not None:
            a = arrays
            self._keep = a
            self.h = lib().svo_index_from_arrays(
                a["buckets"], a["items"], a["gap"], a["padding"], a["bstart"].ctypes.data, a["keys"].ctypes.data,
                a["vals"].ctypes.data, a["length"], a["values_bytes"], a["values"].ctypes.data,
                a["n_chr"], a["chr_end"].ctypes.data)
        else:
            self.h = lib().svo_index_open(prefix.encode())
        if not self.h:
            raise IOError("oracle: cannot load index %s" % prefix)
        nb, items, gap, pad, nchr = (ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int(),
                                     ctypes.c_int(), ctypes.c_uint32())
        lib().svo_index_info(self.h, ctypes.byref(nb), ctypes.byref(items), ctypes.byref(gap),
                             ctypes.byref(pad), ctypes.byref(nchr))
        self.buckets, self.items, self.gap, self.padding, self.n_chr = (
            nb.value, items.value, gap.value, pad.value, nchr.value)

    def prefill(self, keys, block=0):
        """prefill_votes (cell-counts.c:432-491) per key: (bucket-local first item, run length)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        first = np.empty(len(keys), np.uint32)
        count = np.empty(len(keys), np.uint32)
        lib().svo_prefill(self.h, int(block), keys.ctypes.data, len(keys), first.ctypes.data, count.ctypes.data)
        return first, count

    def close(self):
        if self.h:
            lib().svo_index_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def vote(self, params, r1, r2=None, threads=None):
        """-> (mapping[n, ends, multi_best], subjunc or None, big_margin or None, stats[3])"""
        n = len(r1)
        ends = 2 if r2 is not None else 1
        mb = params.multi_best
        out = np.zeros((n, ends, mb), dtype=MAPPING_DTYPE)
        jout = np.zeros((n, ends, mb), dtype=SUBJUNC_DTYPE) if params.do_breakpoint_detection else None
        bm = (np.zeros((n, ends, BIG_MARGIN_WORDS), dtype=np.uint16)
              if params.do_big_margin_filtering_for_junctions else None)
        st = np.zeros(3, dtype=np.uint64)
        s1 = r1.struct()
        s2 = r2.struct() if r2 is not None else None
        rc = lib().svo_vote_batch(
            self.h, ctypes.byref(params), ctypes.byref(s1),
            ctypes.byref(s2) if s2 is not None else None,
            out.ctypes.data, jout.ctypes.data if jout is not None else None,
            bm.ctypes.data if bm is not None else None,
            threads or os.cpu_count() or 1, st.ctypes.data)
        if rc != 0:
            raise RuntimeError("svo_vote_batch failed: %d" % rc)
        return out, jout, bm, st

    def fragile(self, params, r1, r2=None):
        """svo_fragile_batch: the fragile junction voting windows (svg_fragile_batch's form)."""
        from subread_amd.abi import SvgFragileResult
        s1 = r1.struct()
        s2 = r2.struct() if r2 is not None else None
        res = SvgFragileResult()
        rc = lib().svo_fragile_batch(self.h, ctypes.byref(params), ctypes.byref(s1),
                                     ctypes.byref(s2) if s2 is not None else None, ctypes.byref(res))
        if rc != 0:
            raise RuntimeError("svo_fragile_batch failed: %d" % rc)
        try:
            return res.arrays()
        finally:
            lib().svo_fragile_free(ctypes.byref(res))

    def long_vote(self, reads, threads=None):
        """svo_long_vote_batch: sublong's voting step restated (svg_long_vote_batch's form)
        -> (vstart, votes, order)."""
        from subread_amd.abi import SvgLongResult
        s = reads.struct()
        res = SvgLongResult()
        rc = lib().svo_long_vote_batch(self.h, ctypes.byref(s), int(threads or os.cpu_count() or 1), ctypes.byref(res))
        if rc != 0:
            raise RuntimeError("svo_long_vote_batch failed: %d" % rc)
        try:
            return res.arrays()
        finally:
            lib().svo_long_free(ctypes.byref(res))
