"""subread_amd -- MI355X-native seed-and-vote hot path of Subread (subread-align / subjunc).

The product is the C-ABI shared library ``subread_amd/lib/libsubread_amd.so``
(include/subread_vote.h): host C (index loader, format-exact index builder,
read simulator) + hand-written HIP kernels for gfx950.  This module is a thin
ctypes wrapper used by the tests and bench.py.

There is no CPU fallback anywhere in this package: if the library is missing,
or the GPU is missing when a vote is requested, the call raises.
"""
import ctypes
import os
import subprocess

import numpy as np

from .abi import (MAPPING_DTYPE, SUBJUNC_DTYPE, BIG_MARGIN_WORDS, ERRORS, PROGRAM_ALIGN,
                  PROGRAM_SUBJUNC, SvgParams, SvgReads, SvgPackedReads, SvgIndexInfo, SvgBatchStats, ReadBatch,
                  SvgFragileResult,
                  PackedBatch, default_params, read_fastq)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVG_LIB") or os.path.join(HERE, "lib", "libsubread_amd.so")
CSRC = os.path.join(HERE, "csrc")

# every symbol include/subread_vote.h declares
EXPORTS = [
    "svg_params_default", "svg_index_open", "svg_index_close", "svg_index_get_info",
    "svg_vote_batch", "svg_vote_batch_device", "svg_set_stats", "svg_get_stats",
    "svg_last_error", "svg_abi_version", "svg_build_index", "svg_sim_genome",
    "svg_sim_repeats", "svg_sim_reads", "svg_index_build", "svg_index_build_mem", "svg_index_export",
    "svg_set_max_read_length", "svg_sim_pairs", "svg_set_timing", "svg_get_timing",
    "svg_get_kernel_timing", "svg_device_status", "svg_pack_reads", "svg_vote_batch_packed",
    "svg_vote_batch_packed_device", "svg_probe_keys", "svg_probe_keys_device", "svg_host_threads",
    "svg_fragile_batch", "svg_fragile_free", "svg_set_option", "svg_get_option",
    "svg_host_placement", "svg_host_alloc", "svg_host_free", "svg_cpulist_parse",
    # sublong's voting step (include/subread_long.h)
    "svg_long_vote_batch", "svg_long_free",
    # host post-vote events (include/subread_events.h)
    "svg_event_params_default", "svg_genome_arrays_open", "svg_genome_arrays_close", "svg_events_create",
    "svg_events_destroy", "svg_events_add_batch", "svg_events_merge", "svg_events_count", "svg_events_get",
    "svg_events_anti_support", "svg_events_add_batch2", "svg_events_remove_neighbour", "svg_events_load",
    "svg_events_add_windows", "svg_events_load_sites", "svg_index_open_devices",
    # SAM / BAM emission (include/subread_sam.h)
    "svg_sam_writer_open", "svg_sam_writer_close", "svg_sam_writer_begin_chunk", "svg_sam_writer_put",
    "svg_sam_writer_pending", "svg_sam_writer_failed", "svg_sam_format", "svg_sam_writer_put_block",
    "svg_sam_writer_open_bam", "svg_sam_writer_is_bam", "svg_bam_format",
    # iteration two (include/subread_realign.h)
    "svg_realign_params_default", "svg_realign_create", "svg_realign_destroy", "svg_realign_set_events",
    "svg_realign_get_events", "svg_realign_set_tlen_state", "svg_realign_get_tlen_state", "svg_realign_chunk",
    "svg_genome_arrays_contigs", "svg_genome_arrays_wrap",
]

_lib = None


class SvgError(RuntimeError):
    pass


def build(arch="gfx950", quiet=True):
    """Compile libsubread_amd.so in-tree (hipcc --offload-arch=gfx950)."""
    r = subprocess.run(["make", "-C", CSRC, "ARCH=" + arch, "-j8"], capture_output=True, text=True)
    if r.returncode != 0:
        raise SvgError("build of libsubread_amd.so failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])
    if not quiet:
        print(r.stdout)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SvgError("libsubread_amd.so not built (run __graft_entry__.build() or make -C subread_amd/csrc)")
        # one HIP runtime per process: when PyTorch is present, let it load its HIP runtime first
        # so that this library binds to the same one (device buffers are shared with torch)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
        L.svg_params_default.argtypes = [vp, i32, i32]
        L.svg_index_open.argtypes = [ctypes.c_char_p, i32, ctypes.POINTER(vp)]
        L.svg_index_open.restype = i32
        L.svg_index_open_devices.argtypes = [ctypes.c_char_p, vp, i32, vp]
        L.svg_index_open_devices.restype = i32
        L.svg_index_close.argtypes = [vp]
        L.svg_index_get_info.argtypes = [vp, vp]
        L.svg_vote_batch.argtypes = [vp] * 7
        L.svg_vote_batch.restype = i32
        L.svg_vote_batch_device.argtypes = [vp] * 8
        L.svg_vote_batch_device.restype = i32
        L.svg_set_stats.argtypes = [vp, i32]
        L.svg_get_stats.argtypes = [vp, vp]
        L.svg_set_timing.argtypes = [vp, i32]
        L.svg_set_timing.restype = i32
        L.svg_get_timing.argtypes = [vp, vp, vp, vp, vp]
        L.svg_get_timing.restype = i32
        L.svg_get_kernel_timing.argtypes = [vp, vp, vp]
        L.svg_get_kernel_timing.restype = i32
        L.svg_set_max_read_length.argtypes = [vp, i32]
        L.svg_set_max_read_length.restype = i32
        L.svg_device_status.argtypes = [vp]
        L.svg_device_status.restype = i32
        L.svg_pack_reads.argtypes = [vp, u64, vp, vp, vp, i32]
        L.svg_pack_reads.restype = ctypes.c_int64
        L.svg_vote_batch_packed.argtypes = [vp] * 7
        L.svg_vote_batch_packed.restype = i32
        L.svg_vote_batch_packed_device.argtypes = [vp] * 8
        L.svg_vote_batch_packed_device.restype = i32
        L.svg_probe_keys.argtypes = [vp, i32, vp, u64, vp, vp]
        L.svg_probe_keys.restype = i32
        L.svg_probe_keys_device.argtypes = [vp, i32, vp, u64, vp, vp, vp]
        L.svg_probe_keys_device.restype = i32
        L.svg_last_error.restype = ctypes.c_char_p
        L.svg_host_threads.restype = i32
        L.svg_sam_writer_open.argtypes = [vp, ctypes.POINTER(vp)]
        L.svg_sam_writer_open.restype = i32
        L.svg_sam_writer_close.argtypes = [vp]
        L.svg_sam_writer_close.restype = i32
        L.svg_sam_writer_begin_chunk.argtypes = [vp, ctypes.c_int64]
        L.svg_sam_writer_begin_chunk.restype = i32
        L.svg_sam_writer_put.argtypes = [vp, ctypes.c_int64, i32, i32, vp, ctypes.c_size_t]
        L.svg_sam_writer_put.restype = i32
        L.svg_sam_writer_put_block.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_size_t]
        L.svg_sam_writer_put_block.restype = i32
        L.svg_sam_writer_pending.argtypes = [vp]
        L.svg_sam_writer_pending.restype = ctypes.c_int64
        L.svg_sam_writer_failed.argtypes = [vp]
        L.svg_sam_writer_failed.restype = i32
        L.svg_sam_format.argtypes = [vp, vp, ctypes.c_size_t]
        L.svg_sam_format.restype = ctypes.c_int64
        L.svg_host_placement.argtypes = [i32, vp, vp]
        L.svg_host_placement.restype = i32
        L.svg_host_alloc.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
        L.svg_host_alloc.restype = i32
        L.svg_host_free.argtypes = [vp]
        L.svg_cpulist_parse.argtypes = [ctypes.c_char_p, vp, i32]
        L.svg_cpulist_parse.restype = i32
        L.svg_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        L.svg_set_option.restype = i32
        L.svg_get_option.argtypes = [ctypes.c_char_p]
        L.svg_get_option.restype = ctypes.c_int64
        L.svg_fragile_batch.argtypes = [vp] * 5
        L.svg_fragile_batch.restype = i32
        L.svg_fragile_free.argtypes = [vp]
        if hasattr(L, "svg_long_vote_batch"):   # (older builds loaded side by side for A/B runs lack it)
            L.svg_long_vote_batch.argtypes = [vp] * 3
            L.svg_long_vote_batch.restype = i32
            L.svg_long_free.argtypes = [vp]
        L.svg_events_add_batch2.argtypes = [vp] * 8 + [u64] + [vp] * 4
        L.svg_events_add_batch2.restype = i32
        L.svg_index_build.argtypes = [ctypes.c_char_p, i32, i32, i32, i32, i32, ctypes.c_char_p, ctypes.POINTER(vp)]
        L.svg_index_build.restype = i32
        L.svg_index_build_mem.argtypes = [vp, vp, vp, ctypes.c_uint32, i32, i32, i32, i32, i32, ctypes.c_char_p,
                                          ctypes.POINTER(vp)]
        L.svg_index_build_mem.restype = i32
        L.svg_index_export.argtypes = [vp] * 6
        L.svg_index_export.restype = i32
        L.svg_build_index.argtypes = [ctypes.c_char_p, ctypes.c_char_p, i32, i32, i32, i32]
        L.svg_build_index.restype = i32
        L.svg_sim_genome.argtypes = [vp, u64, u64]
        L.svg_sim_repeats.argtypes = [vp, u64, u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, u64]
        L.svg_sim_reads.argtypes = [vp, vp, vp, ctypes.c_uint32, u64, u64, i32, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double, u64, vp, vp, vp, vp, i32]
        L.svg_sim_reads.restype = i32
        L.svg_sim_pairs.argtypes = [vp, vp, vp, ctypes.c_uint32, u64, u64, i32, ctypes.c_double, ctypes.c_double,
                                    i32, ctypes.c_double, u64, vp, vp, i32]
        L.svg_sim_pairs.restype = i32
        L.svg_event_params_default.argtypes = [vp]
        L.svg_genome_arrays_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
        L.svg_genome_arrays_open.restype = i32
        L.svg_genome_arrays_close.argtypes = [vp]
        L.svg_genome_arrays_contigs.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), vp, vp]
        L.svg_genome_arrays_contigs.restype = i32
        L.svg_events_create.argtypes = [ctypes.POINTER(vp)]
        L.svg_events_create.restype = i32
        L.svg_events_destroy.argtypes = [vp]
        L.svg_events_add_batch.argtypes = [vp, vp, vp, vp, vp, vp, u64, vp, vp, vp]
        L.svg_events_add_batch.restype = i32
        L.svg_events_merge.argtypes = [vp, vp, i32]
        L.svg_events_merge.restype = i32
        L.svg_events_anti_support.argtypes = [vp, vp, vp, u64, i32, vp]
        L.svg_events_anti_support.restype = i32
        L.svg_events_remove_neighbour.argtypes = [vp]
        L.svg_events_remove_neighbour.restype = i32
        L.svg_events_load.argtypes = [vp, vp, ctypes.c_int64]
        L.svg_events_load.restype = i32
        L.svg_events_count.argtypes = [vp]
        L.svg_events_count.restype = ctypes.c_int64
        L.svg_events_get.argtypes = [vp, vp]
        L.svg_events_get.restype = i32
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        msg = lib().svg_last_error().decode(errors="replace")
        raise SvgError("%s failed: %s (%s)" % (what, ERRORS.get(rc, rc), msg))


def set_option(name, value):
    """svg_set_option: a process-wide implementation option (include/subread_vote.h); none
    changes a record."""
    _check(lib().svg_set_option(str(name).encode(), int(value)), "svg_set_option(%s)" % name)


def get_option(name):
    return int(lib().svg_get_option(str(name).encode()))


class options:
    """Context manager: set options for a block, restore the previous values after it."""

    def __init__(self, **kw):
        self.kw = kw
        self.old = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.old[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *a):
        for k, v in self.old.items():
            set_option(k, v)
        return False


def params_default(program=PROGRAM_ALIGN, paired=False):
    p = SvgParams()
    lib().svg_params_default(ctypes.byref(p), program, 1 if paired else 0)
    return p


def build_index(fasta, prefix, gap=3, memory_mb=8000, force_one_block=False, repeat_threshold=100):
    """Format-exact subread-buildindex: -F => gap=1, -B => force_one_block, -M => memory_mb
    (a genome over the -M budget is split into .NN blocks as the reference splits it)."""
    rc = lib().svg_build_index(str(fasta).encode(), str(prefix).encode(), gap, memory_mb,
                               1 if force_one_block else 0, repeat_threshold)
    _check(rc, "svg_build_index")


class GenomeArrays:
    """svg_genome_arrays: host copy of an index's base arrays (every .NN.b.array) and contig
    table -- what the event search reads (gvindex_get, locate_gene_position)."""

    def __init__(self, prefix):
        h = ctypes.c_void_p()
        _check(lib().svg_genome_arrays_open(str(prefix).encode(), ctypes.byref(h)), "svg_genome_arrays_open")
        self.h = h

    def contigs(self):
        """[(name, length)] as write_sam_headers' @SQ lines give them (svg_genome_arrays_contigs)."""
        n = ctypes.c_uint32()
        _check(lib().svg_genome_arrays_contigs(self.h, ctypes.byref(n), None, None), "svg_genome_arrays_contigs")
        names = (ctypes.c_char_p * max(1, n.value))()
        lens = (ctypes.c_uint32 * max(1, n.value))()
        _check(lib().svg_genome_arrays_contigs(self.h, ctypes.byref(n), names, lens), "svg_genome_arrays_contigs")
        return [(names[i].decode(), int(lens[i])) for i in range(n.value)]

    def close(self):
        if getattr(self, "h", None):
            lib().svg_genome_arrays_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EventTable:
    """svg_events: the indel / junction events of voted reads (include/subread_events.h)."""

    def __init__(self):
        h = ctypes.c_void_p()
        _check(lib().svg_events_create(ctypes.byref(h)), "svg_events_create")
        self.h = h

    def add_batch(self, genome, params, r1, r2, records, first_read=0, event_params=None, quals=None, fragile=None):
        """records = (mapping, subjunc|None, big_margin|None) as VoteIndex.vote returns them;
        mapping's result_flags gain CORE_IS_GAPPED_READ (64) where the reference sets it.
        quals = (q1, q2|None) ReadBatches of quality strings; fragile = (windows, slots) of
        VoteIndex.fragile (subjunc reads > 160 bp): svg_events_add_batch2."""
        out, jout, bm = records
        s1 = r1.struct()
        s2 = r2.struct() if r2 is not None else None
        ep = ctypes.byref(event_params) if event_params is not None else None
        if quals is None and fragile is None:
            rc = lib().svg_events_add_batch(self.h, genome.h, ctypes.byref(params), ep,
                                            ctypes.byref(s1), ctypes.byref(s2) if s2 is not None else None,
                                            int(first_read), out.ctypes.data,
                                            jout.ctypes.data if jout is not None else None,
                                            bm.ctypes.data if bm is not None else None)
            _check(rc, "svg_events_add_batch")
            return
        q1 = quals[0].struct() if quals is not None else None
        q2 = quals[1].struct() if quals is not None and quals[1] is not None else None
        fr = SvgFragileResult.from_arrays(*fragile) if fragile is not None else None
        rc = lib().svg_events_add_batch2(self.h, genome.h, ctypes.byref(params), ep,
                                         ctypes.byref(s1), ctypes.byref(s2) if s2 is not None else None,
                                         ctypes.byref(q1) if q1 is not None else None,
                                         ctypes.byref(q2) if q2 is not None else None,
                                         int(first_read), out.ctypes.data,
                                         jout.ctypes.data if jout is not None else None,
                                         bm.ctypes.data if bm is not None else None,
                                         ctypes.byref(fr) if fr is not None else None)
        _check(rc, "svg_events_add_batch2")

    @classmethod
    def merge(cls, tables):
        """finalise_indel_and_junction_thread over `tables` (in order) -> a new sorted table."""
        t = cls()
        arr = (ctypes.c_void_p * len(tables))(*[x.h.value for x in tables])
        _check(lib().svg_events_merge(t.h, arr, len(tables)), "svg_events_merge")
        return t

    def anti_support(self, params, n_reads, ends, mapping, event_params=None):
        """svg_events_anti_support over a merged table and the batch's mapping records."""
        _check(lib().svg_events_anti_support(self.h, ctypes.byref(params),
                                             ctypes.byref(event_params) if event_params is not None else None,
                                             int(n_reads), int(ends), mapping.ctypes.data), "svg_events_anti_support")

    def load(self, events):
        """svg_events_load: append an EVENT_DTYPE array (entered in the site lists in order)."""
        from .abi import EVENT_DTYPE
        a = np.ascontiguousarray(events).view(EVENT_DTYPE).reshape(-1)
        _check(lib().svg_events_load(self.h, a.ctypes.data if len(a) else None, len(a)), "svg_events_load")

    def remove_neighbour(self):
        """svg_events_remove_neighbour: remove_neighbour (core-indel.c:447) on a merged table."""
        _check(lib().svg_events_remove_neighbour(self.h), "svg_events_remove_neighbour")

    def events(self):
        from .abi import EVENT_DTYPE
        n = lib().svg_events_count(self.h)
        a = np.zeros(max(0, n), dtype=EVENT_DTYPE)
        _check(lib().svg_events_get(self.h, a.ctypes.data if n else None), "svg_events_get")
        return a

    def close(self):
        if getattr(self, "h", None):
            lib().svg_events_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def find_events(genome, params, r1, r2, records, first_read=0, anti_support=True, quals=None, fragile=None,
                remove_neighbour=False):
    """Events of one batch, merged and sorted like the reference's table after the voting step,
    with the anti-supporting read counts of the scan that follows it (and, remove_neighbour=True,
    the redundant neighbours marked removed as the reference does next)."""
    t = EventTable()
    t.add_batch(genome, params, r1, r2, records, first_read, quals=quals, fragile=fragile)
    m = EventTable.merge([t])
    if anti_support:
        m.anti_support(params, len(r1), 2 if r2 is not None else 1, records[0])
    if remove_neighbour:
        m.remove_neighbour()
    ev = m.events()
    t.close()
    m.close()
    return ev


def pack_reads(batch, stride=None, threads=8, alloc=None):
    """svg_pack_reads: ASCII ReadBatch -> PackedBatch.  stride=None packs the reads back to
    back (starts filled in); else read i goes to base i*stride.  `alloc(nbytes, dtype)` may
    supply the arrays (e.g. pinned memory)."""
    n = len(batch)
    if alloc is None:
        alloc = lambda count, dt: np.empty(count, dt)
    if stride is None:
        total = int(batch.lens.astype(np.int64).sum())
        starts = alloc(max(1, n), np.uint64)
    else:
        total = n * int(stride)
        starts = None
    bases = alloc(max(1, (total + 15) // 16), np.uint32)
    xmask = alloc(max(1, (total + 31) // 32), np.uint32)
    s = batch.struct()
    ne = lib().svg_pack_reads(ctypes.byref(s), int(stride or 0), bases.ctypes.data, xmask.ctypes.data,
                              starts.ctypes.data if starts is not None else None, int(threads))
    if ne < 0:
        _check(int(ne), "svg_pack_reads")
    return PackedBatch(bases, xmask if ne > 0 else None, starts[:n] if starts is not None else None,
                       stride or 0, batch.lens)


class _HostMem:
    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        try:
            lib().svg_host_free(ctypes.c_void_p(self.ptr))
        except Exception:
            pass


class VoteIndex:
    """An index resident in HBM of one GPU (svg_index_open / svg_index_build*)."""

    def __init__(self, prefix=None, device=0, _handle=None):
        if _handle is None:
            h = ctypes.c_void_p()
            _check(lib().svg_index_open(str(prefix).encode(), device, ctypes.byref(h)), "svg_index_open")
            _handle = h
        self.h = _handle
        info = SvgIndexInfo()
        lib().svg_index_get_info(self.h, ctypes.byref(info))
        self.info = info

    @classmethod
    def open_devices(cls, prefix, devices):
        """One replica per listed device from one read of the files (svg_index_open_devices)."""
        n = len(devices)
        devs = (ctypes.c_int32 * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        _check(lib().svg_index_open_devices(str(prefix).encode(), devs, n, hs), "svg_index_open_devices")
        return [cls(_handle=ctypes.c_void_p(hs[k])) for k in range(n)]

    @classmethod
    def build(cls, fasta, gap=1, memory_mb=8000, force_one_block=True, repeat_threshold=100, device=0,
              save_prefix=None):
        """Build the index in HBM (GPU builder); optionally also write the reference files."""
        h = ctypes.c_void_p()
        _check(lib().svg_index_build(str(fasta).encode(), gap, memory_mb, 1 if force_one_block else 0,
                                     repeat_threshold, device, save_prefix.encode() if save_prefix else None,
                                     ctypes.byref(h)), "svg_index_build")
        return cls(_handle=h)

    @classmethod
    def build_genome(cls, genome, gap=1, memory_mb=8000, force_one_block=True, repeat_threshold=100, device=0,
                     save_prefix=None):
        """Build from a subread_amd.sim.Genome (in-memory contigs)."""
        n = len(genome.seqs)
        names = (ctypes.c_char_p * n)(*[x.encode() for x in genome.names])
        seqs = (ctypes.c_void_p * n)(*[s.ctypes.data for s in genome.seqs])
        lens = np.array([len(s) for s in genome.seqs], dtype=np.uint64)
        h = ctypes.c_void_p()
        _check(lib().svg_index_build_mem(names, seqs, lens.ctypes.data, n, gap, memory_mb,
                                         1 if force_one_block else 0, repeat_threshold, device,
                                         save_prefix.encode() if save_prefix else None, ctypes.byref(h)),
               "svg_index_build_mem")
        return cls(_handle=h)

    @property
    def n_blocks(self):
        return self.info.n_blocks

    def host_alloc(self, count, dtype=np.uint8):
        """svg_host_alloc: a pinned host numpy array whose pages sit on the NUMA node of this
        index's GPU; freed (svg_host_free) when the array is no longer referenced."""
        dt = np.dtype(dtype)
        nbytes = max(1, int(count) * dt.itemsize)
        p = ctypes.c_void_p()
        _check(lib().svg_host_alloc(self.h, nbytes, ctypes.byref(p)), "svg_host_alloc")
        buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
        buf._owner = _HostMem(p.value)
        return np.ctypeslib.as_array(buf)[:int(count) * dt.itemsize].view(dt)

    def host_placement(self):
        """(NUMA node of the GPU, usable CPUs on it) -- where svg_host_alloc's pages and the
        expansion workers go."""
        node, ncpu = ctypes.c_int(), ctypes.c_int()
        lib().svg_host_placement(self.info.device, ctypes.byref(node), ctypes.byref(ncpu))
        return node.value, ncpu.value

    def export(self):
        """Host copy of the index arrays of block 00 (dict usable by the oracle's from_arrays)."""
        i = self.info
        a = dict(buckets=i.buckets, items=i.items, gap=i.index_gap, padding=i.padding, length=i.array_length,
                 values_bytes=i.array_values_bytes, n_chr=i.n_chromosomes,
                 bstart=np.empty(i.buckets + 1, np.uint32), keys=np.empty(max(1, i.items), np.int16),
                 vals=np.empty(max(1, i.items), np.uint32), values=np.empty(i.array_values_bytes + 64, np.uint8),
                 chr_end=np.empty(max(1, i.n_chromosomes), np.uint32))
        _check(lib().svg_index_export(self.h, a["bstart"].ctypes.data, a["keys"].ctypes.data, a["vals"].ctypes.data,
                                      a["values"].ctypes.data, a["chr_end"].ctypes.data), "svg_index_export")
        return a

    def close(self):
        if getattr(self, "h", None):
            lib().svg_index_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def probe_keys(self, keys, block=0):
        """svg_probe_keys: cellCounts' prefill_votes lookup for a batch of 32-bit subread keys;
        returns (first, count) -- bucket-local index of each key's equal-key run and its length."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        first = np.empty(len(keys), np.uint32)
        count = np.empty(len(keys), np.uint32)
        _check(lib().svg_probe_keys(self.h, int(block), keys.ctypes.data, len(keys), first.ctypes.data,
                                    count.ctypes.data), "svg_probe_keys")
        return first, count

    def fragile(self, params, r1, r2=None):
        """svg_fragile_batch: the fragile junction voting windows of the batch's subjunc reads
        > 160 bp -> (windows, slots) numpy arrays."""
        s1 = r1.struct()
        s2 = r2.struct() if r2 is not None else None
        res = SvgFragileResult()
        rc = lib().svg_fragile_batch(self.h, ctypes.byref(params), ctypes.byref(s1),
                                     ctypes.byref(s2) if s2 is not None else None, ctypes.byref(res))
        _check(rc, "svg_fragile_batch")
        try:
            return res.arrays()
        finally:
            lib().svg_fragile_free(ctypes.byref(res))

    def long_vote(self, reads):
        """svg_long_vote_batch: sublong's voting step (LRMdo_one_voting_read + the copy and location
        sort, longread-mapping.c:552,668,1317) for a LongReads batch -> (vstart, votes, order)."""
        from .abi import SvgLongResult
        s = reads.struct()
        res = SvgLongResult()
        rc = lib().svg_long_vote_batch(self.h, ctypes.byref(s), ctypes.byref(res))
        _check(rc, "svg_long_vote_batch")
        # views over the library's arrays (no copy of the ~24 B per slot); freed with the last view
        return res.views(lambda r: lib().svg_long_free(ctypes.byref(r)))

    def set_max_read_length(self, n):
        _check(lib().svg_set_max_read_length(self.h, int(n)), "svg_set_max_read_length")

    def device_status(self):
        """Wait for queued work; raise SvgError if a read broke the read-length bound."""
        _check(lib().svg_device_status(self.h), "svg_device_status")

    def set_timing(self, on=True):
        _check(lib().svg_set_timing(self.h, 1 if on else 0), "svg_set_timing")

    def timing(self):
        """{probe_ms, vote_ms, probe_launches, vote_launches} summed since set_timing(True)."""
        pm, vm = ctypes.c_double(), ctypes.c_double()
        pl, vl = ctypes.c_int(), ctypes.c_int()
        _check(lib().svg_get_timing(self.h, ctypes.byref(pm), ctypes.byref(vm), ctypes.byref(pl), ctypes.byref(vl)),
               "svg_get_timing")
        return {"probe_ms": pm.value, "vote_ms": vm.value, "probe_launches": pl.value, "vote_launches": vl.value}

    KERNELS = ("probe_kernel", "vote_kernel", "gather_kernel", "lane_kernel")

    def kernel_timing(self):
        """{kernel: (ms, launches)} per kernel kind since set_timing(True)."""
        ms = (ctypes.c_double * 4)()
        n = (ctypes.c_int * 4)()
        _check(lib().svg_get_kernel_timing(self.h, ms, n), "svg_get_kernel_timing")
        return {k: (ms[i], n[i]) for i, k in enumerate(self.KERNELS)}

    def debug_counters(self):
        """Raw device counters of the last batch with stats on (see svg_debug_counters)."""
        c = (ctypes.c_ulonglong * 32)()
        _check(lib().svg_debug_counters(self.h, c), "svg_debug_counters")
        return list(c)

    def set_stats(self, on=True):
        lib().svg_set_stats(self.h, 1 if on else 0)

    def stats(self):
        s = SvgBatchStats()
        lib().svg_get_stats(self.h, ctypes.byref(s))
        return {"probes": s.probes, "bucket_items": s.bucket_items, "hits": s.hits, "results": s.results,
                "deferred": s.deferred}

    def vote(self, params, r1, r2=None, bufs=None):
        """Host buffers in, host records out: (mapping[n,ends,mb], subjunc|None, big_margin|None).
        `bufs` = a previous call's return value of the same shape, reused as the output
        (the reference's bigtable is likewise allocated once and rewritten per chunk)."""
        n = len(r1)
        ends = 2 if r2 is not None else 1
        mb = params.multi_best
        if bufs is not None:
            out, jout, bm = bufs
            if out.shape != (n, ends, mb) or out.dtype != MAPPING_DTYPE:
                raise ValueError("bufs: mapping array of shape %s expected" % ((n, ends, mb),))
            if (jout is None) != (not params.do_breakpoint_detection) or \
               (bm is None) != (not params.do_big_margin_filtering_for_junctions):
                raise ValueError("bufs: subjunc / big-margin arrays do not match the parameters")
            if jout is not None and (jout.shape != (n, ends, mb) or jout.dtype != SUBJUNC_DTYPE):
                raise ValueError("bufs: subjunc array of shape %s expected" % ((n, ends, mb),))
            if bm is not None and (bm.shape != (n, ends, BIG_MARGIN_WORDS) or bm.dtype != np.uint16):
                raise ValueError("bufs: big-margin array of shape %s expected" % ((n, ends, BIG_MARGIN_WORDS),))
        else:
            out = np.zeros((n, ends, mb), dtype=MAPPING_DTYPE)
            jout = np.zeros((n, ends, mb), dtype=SUBJUNC_DTYPE) if params.do_breakpoint_detection else None
            bm = (np.zeros((n, ends, BIG_MARGIN_WORDS), dtype=np.uint16)
                  if params.do_big_margin_filtering_for_junctions else None)
        s1 = r1.struct()
        s2 = r2.struct() if r2 is not None else None
        rc = lib().svg_vote_batch(self.h, ctypes.byref(params), ctypes.byref(s1),
                                  ctypes.byref(s2) if s2 is not None else None,
                                  out.ctypes.data, jout.ctypes.data if jout is not None else None,
                                  bm.ctypes.data if bm is not None else None)
        _check(rc, "svg_vote_batch")
        return out, jout, bm

    def _outputs(self, params, n, ends, bufs):
        mb = params.multi_best
        if bufs is not None:
            return bufs
        out = np.zeros((n, ends, mb), dtype=MAPPING_DTYPE)
        jout = np.zeros((n, ends, mb), dtype=SUBJUNC_DTYPE) if params.do_breakpoint_detection else None
        bm = (np.zeros((n, ends, BIG_MARGIN_WORDS), dtype=np.uint16)
              if params.do_big_margin_filtering_for_junctions else None)
        return out, jout, bm

    def vote_packed(self, params, p1, p2=None, bufs=None):
        """svg_vote_batch_packed: PackedBatch in (host), records out like vote()."""
        n = len(p1)
        out, jout, bm = self._outputs(params, n, 2 if p2 is not None else 1, bufs)
        s1 = p1.struct()
        s2 = p2.struct() if p2 is not None else None
        rc = lib().svg_vote_batch_packed(self.h, ctypes.byref(params), ctypes.byref(s1),
                                         ctypes.byref(s2) if s2 is not None else None,
                                         out.ctypes.data, jout.ctypes.data if jout is not None else None,
                                         bm.ctypes.data if bm is not None else None)
        _check(rc, "svg_vote_batch_packed")
        return out, jout, bm

    def vote_packed_device(self, params, q1, q2, out_ptr, jout_ptr=None, bm_ptr=None, stream=None):
        """svg_vote_batch_packed_device: q* = SvgPackedReads holding device pointers."""
        rc = lib().svg_vote_batch_packed_device(self.h, ctypes.byref(params), ctypes.byref(q1),
                                                ctypes.byref(q2) if q2 is not None else None,
                                                out_ptr, jout_ptr, bm_ptr, stream)
        _check(rc, "svg_vote_batch_packed_device")

    def vote_device(self, params, r1_ptrs, r2_ptrs, out_ptr, jout_ptr=None, bm_ptr=None, stream=None):
        """Device pointers in/out, async on `stream` (int handle or None).
        r*_ptrs = (seq_ptr, offsets_ptr, lens_ptr, n_reads)."""
        def mk(t):
            s = SvgReads()
            s.seq, s.offsets, s.lens, s.n_reads = t
            return s
        s1 = mk(r1_ptrs)
        s2 = mk(r2_ptrs) if r2_ptrs is not None else None
        rc = lib().svg_vote_batch_device(self.h, ctypes.byref(params), ctypes.byref(s1),
                                         ctypes.byref(s2) if s2 is not None else None,
                                         out_ptr, jout_ptr, bm_ptr, stream)
        _check(rc, "svg_vote_batch_device")
