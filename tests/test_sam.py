"""SAM emission (include/subread_sam.h, f2 row): svg_sam_format against the reference's format
string for add_buffered_fragment's SAM lines ("%s\\t%d\\t%s\\t%u\\t%d\\t%s\\t%s\\t%u\\t%d\\t%s\\t%s%s%s\\n",
core.c:1865-1867), and svg_sam_writer's ordering: fragments put out of order from many threads, with
several locations each, leave in fragment order and per-fragment put order, chunk after chunk --
the order add_buffered_fragment's spin enforces (core.c:1855-1881).  The live check is the drop-in
(tests/test_dropin.py at -T 4, tests/test_gpu_dropin.py): stock and drop-in SAM byte-identical."""
import ctypes
import random
import threading

import pytest

import subread_amd as sa


class Rec(ctypes.Structure):
    _fields_ = [("qname", ctypes.c_char_p), ("flag", ctypes.c_int32), ("rname", ctypes.c_char_p),
                ("pos", ctypes.c_uint32), ("mapq", ctypes.c_int32), ("cigar", ctypes.c_char_p),
                ("rnext", ctypes.c_char_p), ("pnext", ctypes.c_uint32), ("tlen", ctypes.c_int32),
                ("seq", ctypes.c_char_p), ("qual", ctypes.c_char_p), ("tags", ctypes.c_char_p)]


def ref_line(f):
    # the reference's format string, as C's printf renders it (%u of an unsigned int, %d of an int)
    tags = f["tags"]
    return b"%s\t%d\t%s\t%d\t%d\t%s\t%s\t%d\t%d\t%s\t%s%s%s\n" % (
        f["qname"], f["flag"], f["rname"], f["pos"], f["mapq"], f["cigar"], f["rnext"], f["pnext"], f["tlen"],
        f["seq"], f["qual"], b"\t" if tags else b"", tags)


def rand_fields(rng):
    return dict(qname=b"r%d" % rng.randrange(10 ** 9), flag=rng.choice([0, 4, 16, 83, 163, 2047]),
                rname=rng.choice([b"*", b"chr1", b"chrUn_KI270302v1"]), pos=rng.choice([0, 1, 4294967295, rng.randrange(2 ** 32)]),
                mapq=rng.choice([0, 1, 40, 255]), cigar=rng.choice([b"*", b"100M", b"3S45M2I50M"]),
                rnext=rng.choice([b"*", b"="]), pnext=rng.randrange(2 ** 32),
                tlen=rng.choice([0, -1, 1, -2147483648, 2147483647, rng.randrange(-10 ** 6, 10 ** 6)]),
                seq=bytes(rng.choice(b"ACGTN") for _ in range(rng.randrange(0, 300))),
                qual=bytes(rng.randrange(33, 75) for _ in range(rng.randrange(0, 300))),
                tags=rng.choice([b"", b"HI:i:1\tNH:i:1\tNM:i:0", b"HI:i:2\tNH:i:3\tRG:Z:x\tNM:i:12"]))


def fmt(f, cap=1 << 16):
    r = Rec(**f)
    buf = ctypes.create_string_buffer(cap)
    n = sa.lib().svg_sam_format(ctypes.byref(r), buf, cap)
    return buf.raw[:n] if n >= 0 else n


def test_sam_format_matches_reference_format_string():
    rng = random.Random(7)
    for _ in range(3000):
        f = rand_fields(rng)
        assert fmt(f) == ref_line(f)


def test_sam_format_reports_overflow():
    f = rand_fields(random.Random(1))
    line = ref_line(f)
    assert fmt(f, len(line)) == line
    assert fmt(f, len(line) - 1) < 0


libc = ctypes.CDLL(None)
libc.fopen.restype = ctypes.c_void_p
libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
libc.fclose.argtypes = [ctypes.c_void_p]
libc.fputs.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


@pytest.mark.parametrize("threads", [1, 8])
def test_sam_writer_orders_fragments_across_threads(tmp_path, threads):
    L = sa.lib()
    rng = random.Random(threads)
    path = str(tmp_path / "out.sam")
    fp = libc.fopen(path.encode(), b"w")
    libc.fputs(b"@HD\tVN:1.0\n", fp)          # the caller's header goes first, through the same FILE*
    w = ctypes.c_void_p()
    assert L.svg_sam_writer_open(fp, ctypes.byref(w)) == 0
    want = [b"@HD\tVN:1.0\n"]
    for chunk in range(3):
        n = rng.randrange(1, 5000)
        assert L.svg_sam_writer_begin_chunk(w, n) == 0
        # fragment -> its locations' texts; unmapped fragments have one location
        frags = []
        for k in range(n):
            locs = [b"c%d f%d loc%d %s\n" % (chunk, k, j, b"x" * rng.randrange(0, 600)) for j in range(rng.choice([1, 1, 1, 2, 3]))]
            frags.append(locs)
            want += locs
        # each worker takes fragments in a shuffled order and puts all locations of one fragment in order
        order = list(range(n))
        rng.shuffle(order)
        parts = [order[t::threads] for t in range(threads)]
        errs = []

        def work(ks):
            for k in ks:
                for j, t in enumerate(frags[k]):
                    rc = L.svg_sam_writer_put(w, k, j, len(frags[k]), t, len(t))
                    if rc:
                        errs.append((k, j, rc))
        th = [threading.Thread(target=work, args=(p,)) for p in parts]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs
        assert L.svg_sam_writer_pending(w) == 0
    # a fragment already written is refused
    assert L.svg_sam_writer_put(w, 0, 0, 1, b"x\n", 2) != 0
    assert L.svg_sam_writer_failed(w) == 0
    assert L.svg_sam_writer_close(w) == 0
    libc.fclose(fp)
    assert open(path, "rb").read() == b"".join(want)


@pytest.mark.parametrize("threads", [1, 8])
def test_sam_writer_blocks_and_big_chunks(tmp_path, threads):
    """svg_sam_writer_put_block (the runs of fragments svg_realign_chunk's workers put) mixed with
    single puts, chunks of more than 8 MB from 8 threads, one fragment larger than 4 MB (the
    staging buffer's growth) and empty fragments (--ignoreUnmapped writes nothing for a fragment):
    fragment order, chunk after chunk."""
    L = sa.lib()
    rng = random.Random(100 + threads)
    path = str(tmp_path / "big.sam")
    fp = libc.fopen(path.encode(), b"w")
    w = ctypes.c_void_p()
    assert L.svg_sam_writer_open(fp, ctypes.byref(w)) == 0
    want = []
    for chunk in range(2):
        n = 6000
        assert L.svg_sam_writer_begin_chunk(w, n) == 0
        texts = []
        for k in range(n):
            if k == 1234 and chunk == 1:
                t = b"huge %d " % k + b"y" * (5 << 20) + b"\n"
            elif k % 97 == 0:
                t = b""
            else:
                t = b"c%d f%d %s\n" % (chunk, k, b"x" * rng.randrange(1000, 3000))
            texts.append(t)
            want.append(t)
        # runs of 1..300 fragments, put as blocks (a run of one as a single put), in shuffled order
        runs, k = [], 0
        while k < n:
            m = min(n - k, rng.randrange(1, 300))
            runs.append((k, m))
            k += m
        rng.shuffle(runs)
        parts = [runs[t::threads] for t in range(threads)]
        errs = []

        def work(rs):
            for (b, m) in rs:
                txt = b"".join(texts[b:b + m])
                if m == 1 and txt:
                    rc = L.svg_sam_writer_put(w, b, 0, 1, txt, len(txt))
                else:
                    rc = L.svg_sam_writer_put_block(w, b, m, txt, len(txt))
                if rc:
                    errs.append((b, m, rc))
        th = [threading.Thread(target=work, args=(p,)) for p in parts]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs
        assert L.svg_sam_writer_pending(w) == 0
    assert L.svg_sam_writer_failed(w) == 0
    assert L.svg_sam_writer_close(w) == 0
    libc.fclose(fp)
    got = open(path, "rb").read()
    assert len(got) > 16 << 20
    assert got == b"".join(want)


def test_sam_writer_reports_a_failed_write():
    """A short write (a full device) sets svg_sam_writer_failed and fails the put that wrote it and
    the close -- the reference's output_sam_is_full (core.c:1869-1871)."""
    import os
    if not os.path.exists("/dev/full"):
        pytest.skip("no /dev/full")
    L = sa.lib()
    fp = libc.fopen(b"/dev/full", b"w")
    w = ctypes.c_void_p()
    assert L.svg_sam_writer_open(fp, ctypes.byref(w)) == 0
    assert L.svg_sam_writer_begin_chunk(w, 3) == 0
    t = b"x" * (3 << 20) + b"\n"
    rcs = [L.svg_sam_writer_put(w, k, 0, 1, t, len(t)) for k in range(3)]
    assert any(rcs) or L.svg_sam_writer_failed(w)
    assert L.svg_sam_writer_failed(w) == 1
    assert L.svg_sam_writer_close(w) != 0
    libc.fclose(fp)
