"""ctypes mirror of include/subread_vote.h (the C ABI of the vote path).

Record layouts are byte-identical to the reference's bigtable structs:
mapping_result_t (core.h:350-370, 68 B) and subjunc_result_t (core.h:397-410,
16 B).  Parameter defaults follow the reference's own order of precedence:
init_global_context (core-indel.c:4399-4538), parse_opts_aligner /
parse_opts_subjunc (core-interface-aligner.c:256-300, core-interface-subjunc.c:255-290,
:671), then load_global_context's overrides (core.c:4075-4094).
"""
import ctypes
import numpy as np

MAX_READ_LENGTH = 1210
BIG_MARGIN_WORDS = 9
NEGATIVE_STRAND_FLAG = 8
PROGRAM_ALIGN = 0
PROGRAM_SUBJUNC = 1

ERRORS = {0: "OK", -1: "SVG_E_ARG", -2: "SVG_E_IO", -3: "SVG_E_FORMAT",
          -4: "SVG_E_UNSUPPORTED", -5: "SVG_E_DEVICE", -6: "SVG_E_NOMEM"}

MAPPING_DTYPE = np.dtype([
    ("selected_position", "<u4"),
    ("result_flags", "<i2"),
    ("read_length", "<i2"),
    ("selected_votes", "<i2"),
    ("used_subreads_in_vote", "<i2"),
    ("noninformative_subreads_in_vote", "u1"),
    ("indels_in_confident_coverage", "i1"),
    ("is_fully_covered", "i1"),
    ("_pad0", "u1"),
    ("selected_indel_record", "<i2", (22,)),
    ("confident_coverage_start", "<u2"),
    ("confident_coverage_end", "<u2"),
    ("subread_quality", "<i2"),
    ("_pad1", "<u2"),
])
assert MAPPING_DTYPE.itemsize == 68

# svg_event (include/subread_events.h): chromosome_event_t, core.h:274-346, bases decoded
EVENT_DTYPE = np.dtype([
    ("small_side", "<u4"), ("large_side", "<u4"), ("indel_length", "<i2"),
    ("junction_flanking_left", "<i2"), ("junction_flanking_right", "<i2"),
    ("indel_at_junction", "i1"), ("is_negative_strand", "i1"), ("is_strand_jumped", "i1"),
    ("is_donor_found_or_annotation", "i1"), ("small_side_increasing_coordinate", "i1"),
    ("large_side_increasing_coordinate", "i1"), ("connected_next_event_distance", "i1"),
    ("connected_previous_event_distance", "i1"), ("supporting_reads", "<u2"), ("anti_supporting_reads", "<u2"),
    ("final_counted_reads", "<u2"), ("final_reads_mismatches", "<u2"), ("event_type", "u1"),
    ("inserted_len", "u1"), ("critical_read_id", "<u8"), ("event_quality", "<f4"),
    ("critical_supporting_reads", "<i4"), ("inserted_bases", "S40"),
], align=True)
assert EVENT_DTYPE.itemsize == 88

EVENT_INDEL, EVENT_JUNCTION, EVENT_FUSION = 8, 64, 128


class SvgEventParams(ctypes.Structure):
    _fields_ = [("dp_penalty_create_gap", ctypes.c_int32), ("dp_penalty_extend_gap", ctypes.c_int32),
                ("dp_match_score", ctypes.c_int32), ("dp_mismatch_penalty", ctypes.c_int32),
                ("report_multi_mapping_reads", ctypes.c_int32), ("quality_base", ctypes.c_int32),
                ("maximise_sensitivity_indel", ctypes.c_int32)]


SUBJUNC_DTYPE = np.dtype([
    ("split_point", "<i2"),
    ("minor_votes", "<i2"),
    ("double_indel_offset", "i1"),
    ("indel_at_junction", "i1"),
    ("small_side_increasing_coordinate", "i1"),
    ("large_side_increasing_coordinate", "i1"),
    ("minor_position", "<u4"),
    ("minor_coverage_start", "<u2"),
    ("minor_coverage_end", "<u2"),
])
assert SUBJUNC_DTYPE.itemsize == 16

_PARAM_FIELDS = [
    "total_subreads", "min_votes_first", "min_votes_second", "max_indel_length",
    "multi_best", "top_scores", "max_vote_simples", "max_vote_combinations",
    "max_vote_number_cutoff", "min_pair_distance", "max_pair_distance",
    "reverse_r1", "reverse_r2", "do_breakpoint_detection",
    "do_big_margin_filtering_for_junctions", "big_margin_record_size",
    "maximum_intron_length", "prefer_donor_receptor_junctions",
    "check_donor_at_junctions", "max_insertion_at_junctions", "more_accurate_fusions",
]


class SvgParams(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int32) for f in _PARAM_FIELDS]

    def as_dict(self):
        return {f: getattr(self, f) for f in _PARAM_FIELDS}


class SvgReads(ctypes.Structure):
    _fields_ = [
        ("seq", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("lens", ctypes.c_void_p),
        ("n_reads", ctypes.c_uint64),
    ]


class SvgPackedReads(ctypes.Structure):
    _fields_ = [
        ("bases", ctypes.c_void_p),
        ("xmask", ctypes.c_void_p),
        ("starts", ctypes.c_void_p),
        ("stride", ctypes.c_uint64),
        ("lens", ctypes.c_void_p),
        ("n_reads", ctypes.c_uint64),
    ]


class SvgIndexInfo(ctypes.Structure):
    _fields_ = [
        ("items", ctypes.c_uint64),
        ("buckets", ctypes.c_uint32),
        ("index_gap", ctypes.c_int32),
        ("padding", ctypes.c_int32),
        ("array_length", ctypes.c_uint32),
        ("n_chromosomes", ctypes.c_uint32),
        ("device_bytes", ctypes.c_uint64),
        ("device", ctypes.c_int32),
        ("array_values_bytes", ctypes.c_uint32),
        ("n_blocks", ctypes.c_int32),
    ]


# svg_fragile_window / svg_fragile_slot (include/subread_vote.h): fragile junction voting windows
FRAGILE_WINDOW_DTYPE = np.dtype([
    ("read", "<u4"), ("block", "u1"), ("strand", "u1"), ("end", "u1"), ("window", "u1"),
    ("start", "<u2"), ("length", "<u2"), ("junction", "u1"), ("gtag", "u1"), ("n_slots", "<u2"),
    ("small_side", "<u4"), ("large_side", "<u4"), ("first_slot", "<u4")])
FRAGILE_SLOT_DTYPE = np.dtype([("position", "<u4"), ("rec", "<i2", (9,)), ("_pad", "<u2")])
assert FRAGILE_WINDOW_DTYPE.itemsize == 28 and FRAGILE_SLOT_DTYPE.itemsize == 24


class SvgFragileResult(ctypes.Structure):
    _fields_ = [("n_windows", ctypes.c_uint64), ("n_slots", ctypes.c_uint64),
                ("windows", ctypes.c_void_p), ("slots", ctypes.c_void_p)]

    def arrays(self):
        """Copies of the windows and slots as numpy structured arrays."""
        w = np.zeros(self.n_windows, dtype=FRAGILE_WINDOW_DTYPE)
        sl = np.zeros(self.n_slots, dtype=FRAGILE_SLOT_DTYPE)
        if self.n_windows:
            ctypes.memmove(w.ctypes.data, self.windows, w.nbytes)
        if self.n_slots:
            ctypes.memmove(sl.ctypes.data, self.slots, sl.nbytes)
        return w, sl

    @classmethod
    def from_arrays(cls, w, sl):
        """A result struct over numpy arrays (keep them alive while it is used)."""
        r = cls()
        r.n_windows, r.n_slots = len(w), len(sl)
        r.windows = w.ctypes.data if len(w) else None
        r.slots = sl.ctypes.data if len(sl) else None
        return r


# svg_long_vote (include/subread_long.h): one used slot of sublong's LRMgene_vote_t
LONG_VOTE_DTYPE = np.dtype([("pos", "<u4"), ("coverage_start", "<u4"), ("coverage_end", "<u4"),
                            ("votes", "<u2"), ("negative", "u1"), ("_pad", "u1"), ("slot", "<u4")])
assert LONG_VOTE_DTYPE.itemsize == 20


class LongReads:
    """sublong's reads (svg_long_reads): concatenated ASCII, u64 offsets, u32 lengths."""

    def __init__(self, seq, offsets, lens):
        self.seq = np.ascontiguousarray(seq, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.lens = np.ascontiguousarray(lens, dtype=np.uint32)
        assert self.offsets.shape == self.lens.shape

    @classmethod
    def from_list(cls, reads):
        reads = [r.encode() if isinstance(r, str) else bytes(r) for r in reads]
        lens = np.array([len(r) for r in reads], dtype=np.uint32)
        offs = np.zeros(len(reads), dtype=np.uint64)
        if len(reads) > 1:
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        seq = np.frombuffer(b"".join(reads), dtype=np.uint8) if reads else np.zeros(0, np.uint8)
        return cls(seq, offs, lens)

    def __len__(self):
        return int(self.lens.shape[0])

    def read(self, i):
        o = int(self.offsets[i])
        return bytes(self.seq[o:o + int(self.lens[i])])

    def slice(self, a, b):
        return LongReads(self.seq, self.offsets[a:b], self.lens[a:b])

    def struct(self):
        s = SvgLongReads()
        s.seq = self.seq.ctypes.data if self.seq.size else None
        s.offsets = self.offsets.ctypes.data if len(self) else None
        s.lens = self.lens.ctypes.data if len(self) else None
        s.n_reads = len(self)
        s._keep = self
        return s


class SvgLongReads(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("n_reads", ctypes.c_uint64)]


class _Owner:
    """Frees a library-owned result once every numpy view of it is gone."""

    def __init__(self, res, free):
        self.res, self.free, self.n = res, free, 3

    def drop(self):
        self.n -= 1
        if self.n == 0:
            self.free(self.res)


class SvgLongResult(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_uint64), ("vstart", ctypes.c_void_p), ("votes", ctypes.c_void_p),
                ("order", ctypes.c_void_p)]

    def views(self, free):
        """(vstart, votes, order) numpy arrays over the library's buffers, no copy; `free(result)`
        runs when the last of them is garbage-collected."""
        import weakref
        n = int(self.n_reads)
        vs = np.ctypeslib.as_array(ctypes.cast(self.vstart, ctypes.POINTER(ctypes.c_uint64)), (n + 1,))
        k = int(vs[-1])
        if k == 0:
            out = (vs.copy(), np.zeros(0, LONG_VOTE_DTYPE), np.zeros(0, np.uint32))
            free(self)
            return out
        raw = np.ctypeslib.as_array(ctypes.cast(self.votes, ctypes.POINTER(ctypes.c_uint8)), (k * 20,))
        v = raw.view(LONG_VOTE_DTYPE)
        o = np.ctypeslib.as_array(ctypes.cast(self.order, ctypes.POINTER(ctypes.c_uint32)), (k,))
        owner = _Owner(self, free)
        for a in (vs, raw, o):
            weakref.finalize(a, owner.drop)
        return vs, v, o

    def arrays(self):
        """Copies: (vstart[n+1] u64, votes LONG_VOTE_DTYPE, order u32)."""
        n = int(self.n_reads)
        vs = np.zeros(n + 1, np.uint64)
        if self.vstart:
            ctypes.memmove(vs.ctypes.data, self.vstart, vs.nbytes)
        k = int(vs[-1])
        v = np.zeros(k, LONG_VOTE_DTYPE)
        o = np.zeros(k, np.uint32)
        if k:
            ctypes.memmove(v.ctypes.data, self.votes, v.nbytes)
            ctypes.memmove(o.ctypes.data, self.order, o.nbytes)
        return vs, v, o


class SvgBatchStats(ctypes.Structure):
    _fields_ = [
        ("probes", ctypes.c_uint64),
        ("bucket_items", ctypes.c_uint64),
        ("hits", ctypes.c_uint64),
        ("results", ctypes.c_uint64),
        ("deferred", ctypes.c_uint64),
    ]


def default_params(program=PROGRAM_ALIGN, paired=False, **overrides):
    """Python mirror of svg_params_default() (same values, same precedence)."""
    p = SvgParams()
    # init_global_context, core-indel.c:4399-4538
    p.total_subreads = 10
    p.min_votes_first = 3
    p.min_votes_second = 1
    p.max_indel_length = 5
    p.top_scores = 3
    p.min_pair_distance = 50
    p.max_pair_distance = 600
    p.reverse_r1 = 0
    p.reverse_r2 = 1
    p.do_breakpoint_detection = 0
    p.do_big_margin_filtering_for_junctions = 0
    p.big_margin_record_size = 9
    p.maximum_intron_length = 500000
    p.prefer_donor_receptor_junctions = 1
    p.check_donor_at_junctions = 1
    p.max_insertion_at_junctions = 0
    p.more_accurate_fusions = 1
    if program == PROGRAM_SUBJUNC:
        # parse_opts_subjunc, core-interface-subjunc.c:268-282
        p.do_breakpoint_detection = 1
        p.total_subreads = 14
        p.min_votes_first = 1
        p.min_votes_second = 1
        p.do_big_margin_filtering_for_junctions = 1
    # more_accurate_fusions only survives with fusion / long-del detection
    # (core-interface-aligner.c:648, core-interface-subjunc.c:671)
    p.more_accurate_fusions = 0
    # load_global_context overrides, core.c:4075-4084 (reported_multi_best_reads = 1)
    p.max_vote_combinations = 3
    p.multi_best = 3
    p.max_vote_simples = 64 if paired else 3
    p.max_vote_number_cutoff = 2
    for k, v in overrides.items():
        setattr(p, k, int(v))
    return p


class ReadBatch:
    """Concatenated ASCII reads + offsets + lengths, kept alive for ctypes."""

    def __init__(self, seq, offsets, lens):
        self.seq = np.ascontiguousarray(seq, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.lens = np.ascontiguousarray(lens, dtype=np.uint16)
        assert self.offsets.shape == self.lens.shape

    @classmethod
    def from_list(cls, reads):
        reads = [r.encode() if isinstance(r, str) else bytes(r) for r in reads]
        lens = np.array([len(r) for r in reads], dtype=np.uint16)
        offs = np.zeros(len(reads), dtype=np.uint64)
        if len(reads) > 1:
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        seq = np.frombuffer(b"".join(reads), dtype=np.uint8) if reads else np.zeros(0, np.uint8)
        return cls(seq, offs, lens)

    @classmethod
    def fixed(cls, seq2d):
        """Reads of one length: seq2d is an (n, L) uint8 array."""
        seq2d = np.ascontiguousarray(seq2d, dtype=np.uint8)
        n, L = seq2d.shape
        return cls(seq2d.reshape(-1), np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint16))

    def __len__(self):
        return int(self.lens.shape[0])

    def slice(self, a, b):
        return ReadBatch(self.seq, self.offsets[a:b], self.lens[a:b])

    def read(self, i):
        o = int(self.offsets[i])
        return bytes(self.seq[o:o + int(self.lens[i])])

    def struct(self):
        s = SvgReads()
        s.seq = self.seq.ctypes.data
        s.offsets = self.offsets.ctypes.data
        s.lens = self.lens.ctypes.data
        s.n_reads = len(self)
        return s


PACK_CODE = np.full(256, 3, np.uint8)        # base2int, subread.h:238
PACK_CODE[:ord("G")] = 2
PACK_CODE[ord("A")] = 0
PACK_CODE[ord("G")] = 1
PACK_EXCEPTION = np.ones(256, bool)           # complements to 'N' in reverse_read (input-files.c:1111)
PACK_EXCEPTION[[ord(c) for c in "ACGTU"]] = False


class PackedBatch:
    """Reads in the 2-bit form of svg_packed_reads (include/subread_vote.h).
    `xmask` is None when every base is A/C/G/T/U; `starts` None means read i at i*stride."""

    def __init__(self, bases, xmask, starts, stride, lens):
        self.bases = np.ascontiguousarray(bases, dtype=np.uint32)
        self.xmask = None if xmask is None else np.ascontiguousarray(xmask, dtype=np.uint32)
        self.starts = None if starts is None else np.ascontiguousarray(starts, dtype=np.uint64)
        self.stride = int(stride)
        self.lens = np.ascontiguousarray(lens, dtype=np.uint16)

    def __len__(self):
        return int(self.lens.shape[0])

    def struct(self):
        s = SvgPackedReads()
        s.bases = self.bases.ctypes.data
        s.xmask = self.xmask.ctypes.data if self.xmask is not None else None
        s.starts = self.starts.ctypes.data if self.starts is not None else None
        s.stride = self.stride
        s.lens = self.lens.ctypes.data
        s.n_reads = len(self)
        return s

    @classmethod
    def pack_numpy(cls, batch, stride=None):
        """Pure-numpy packer (test cross-check of svg_pack_reads): back to back when
        stride is None, else read i at base i*stride."""
        n = len(batch)
        lens = batch.lens.astype(np.int64)
        if stride is None:
            starts = np.zeros(n, np.uint64)
            if n > 1:
                starts[1:] = np.cumsum(lens[:-1]).astype(np.uint64)
            total = int(lens.sum())
            pos = starts.astype(np.int64)
        else:
            starts = None
            total = n * stride
            pos = np.arange(n, dtype=np.int64) * stride
        codes = np.zeros(total + 32, np.uint8)
        xm = np.zeros(total + 32, bool)
        for i in range(n):
            c = np.frombuffer(batch.read(i), dtype=np.uint8)
            codes[pos[i]:pos[i] + len(c)] = PACK_CODE[c]
            xm[pos[i]:pos[i] + len(c)] = PACK_EXCEPTION[c]
        nw = (total + 15) // 16
        cw = codes[:nw * 16].reshape(nw, 16).astype(np.uint32)
        bases = (cw << (30 - 2 * np.arange(16, dtype=np.uint32))).sum(1, dtype=np.uint64).astype(np.uint32)
        nx = (total + 31) // 32
        xw = xm[:nx * 32].reshape(nx, 32).astype(np.uint64)
        xmask = (xw << (31 - np.arange(32, dtype=np.uint64))).sum(1).astype(np.uint32)
        return cls(bases, xmask if xm.any() else None, starts, stride or 0, batch.lens)


def read_fastq(path):
    """Minimal FASTQ reader (plain or .gz) -> (names, ReadBatch)."""
    import gzip
    op = gzip.open if str(path).endswith(".gz") else open
    names, reads = [], []
    with op(path, "rb") as f:
        while True:
            h = f.readline()
            if not h:
                break
            s = f.readline().rstrip(b"\r\n")
            f.readline()
            f.readline()
            names.append(h[1:].split()[0].decode())
            reads.append(s)
    return names, ReadBatch.from_list(reads)
