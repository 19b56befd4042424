"""CPU: the drop-in binding (integration/do_voting_gpu.c) inside the reference's own
subread-align / subjunc, with the vote answered by the CPU restatement
(oracle/dropin_oracle.c) and iteration two run by the library (svg_realign_chunk,
include/subread_realign.h -- host C, no GPU), gives the stock reference's SAM / VCF / junction
BED / event table byte for byte.  This pins the binding's host logic -- chunk reading, bigtable
layout, big-margin staging, the post-vote tail's text/quality orientation, fragile junction
voting of long subjunc reads, the multi-block run loop, -T > 1 -- and the library's iteration
two (realignment against the event table, candidate choice, SAM fields, event support for the
VCF / BED) apart from the kernels; tests/test_gpu_dropin.py runs the same binding with the GPU
library.  Needs the binaries built from /root/reference (this container; skipped where they
are absent)."""
import os

import numpy as np
import pytest

from tests.common import Case, IndexCache
from tests.dropin import check_case, have


@pytest.fixture(scope="module")
def cache(tmp_path_factory):
    return IndexCache(str(tmp_path_factory.mktemp("dropin_idx")))


@pytest.mark.parametrize("name,threads", [
    ("pe_gapped_errmut", 1),            # PE align, test-err-mut pairs
    ("pe_gapped_errmut", 4),            # the same at -T 4 (iteration two's worker threads)
    ("sj_pe_gapped_junc", 1),           # subjunc PE, junction reads: junction events, XS tags, BED support
    ("sj_pe_gapped_long", 1),           # subjunc PE > 160 bp: fragile junction voting in the binding
    ("sj_pe_mb_long_gappedM6", 1),      # subjunc PE on a 4-block index (block loop)
    ("sj_se_mb_synth_long_fullM1", 1),  # subjunc SE > 160 bp on a 4-block index: fragile windows per block
    ("se_gapped_mixed_n14_I16", 4),     # -n 14 -I 16, N / lowercase / IUPAC, -T 4
    ("se_mb_synth_fullM1", 1),          # SE on a 4-block index: iteration two's value-index choice per record
    ("pe_mb_synth_gappedM1", 1),        # PE on a 2-block index
])
def test_oracle_dropin_matches_stock_reference(name, threads, cache, tmp_path):
    c = Case(name)
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "oracle-dropin", threads)
    assert rep["mapped"] > 0


@pytest.mark.parametrize("name,threads", [("pe_gapped_errmut", 4), ("sj_pe_gapped_long", 1),
                                          ("se_gapped_mixed_n14_I16", 2)])   # reads holding NUL bytes
def test_votetime_harness_matches_stock_reference(name, threads, cache, tmp_path):
    """The CPU-baseline timing harness (oracle/ref_votetime.c: reads parsed before the clock,
    served from memory) changes nothing the aligner writes."""
    c = Case(name)
    if not have(c.meta["program"], "votetime"):
        pytest.skip("reference timing binaries not built (make -C oracle votetime)")
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "votetime", threads)
    assert rep["mapped"] > 0


@pytest.mark.parametrize("name,threads", [("pe_gapped_errmut", 4), ("se_gapped_mixed_n14_I16", 2)])
def test_votetime_chunked_mode_votes_every_read(name, threads, cache, tmp_path):
    """bench.py's cpu_baseline timing of the reference (SVG_REF_CHUNK: the reads in chunks of one
    process, iteration two skipped): one clock line per chunk, every read voted once, and the
    vote records of the chunks, one after another, are the golden records of the case."""
    import math
    import re
    from tests.dropin import fastq_pair, run, case_extra
    c = Case(name)
    if not have(c.meta["program"], "votetime"):
        pytest.skip("reference timing binaries not built (make -C oracle votetime)")
    n = len(c.r1)
    size = math.ceil(n / 3)
    f1, f2 = fastq_pair(str(tmp_path), c.name, c.r1, c.r2)
    out = str(tmp_path / "vt.sam")
    r = run(c.meta["program"], "votetime", cache.get(c.index_key), f1, f2, out, threads, case_extra(c),
            env={"SVG_REF_CHUNK": str(size), "SVG_REF_VOTETIME": "1"})
    lines = re.findall(r"SVG_REF_CHUNK_VOTING_S (\d+) ([0-9.]+) (\d+)", r.stderr)
    assert [int(x[0]) for x in lines] == list(range(math.ceil(n / size)))
    assert [int(x[2]) for x in lines] == [min(size, n - k * size) for k in range(len(lines))]
    assert all(float(x[1]) > 0 for x in lines)
    votes = np.fromfile(out + ".votes", dtype=np.uint8)
    assert votes.size == c.expected.size and (votes.reshape(c.expected.shape) == c.expected).all()


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


@pytest.mark.parametrize("trim", [(), ("--trim5", "3", "--trim3", "2")])
def test_oracle_dropin_fastq_layouts_match_stock(trim, cache, tmp_path):
    """The binding's plain-FASTQ parse (fq_next_read: geinput_next_read_trim's FASTQ branch,
    input-files.c:982-1093, one stdio lock per read) against the reference's own parser inside
    the stock aligner: read names cut at the first blank or tab after their first character,
    empty names, blank lines between and inside records, '+' lines with text, CR bytes kept, a
    read longer than MAX_READ_LENGTH cut to it, reads of every length, 5'/3' trimming -- the
    same SAM / VCF byte for byte, with two threads (the chunk's reads are fetched once and
    served to the later passes from the binding's cache)."""
    from tests import dropin
    c = Case("pe_gapped_errmut")
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    fq = str(tmp_path / "r.fq")
    with open(fq, "wb") as f:
        for i in range(len(c.r1)):
            s = c.r1.read(i)
            q = bytes(33 + (i * 5 + k * 11) % 41 for k in range(len(s)))
            k = i % 9
            if k == 0:
                name = b"r%d extra comment" % i
            elif k == 1:
                name = b"r%d\tBX:Z:ACGT" % i
            elif k == 2:
                name = b" r%d" % i             # blank at position 0 is kept (the cut starts at 1)
            elif k == 3:
                name = b"x"
            else:
                name = b"r%d" % i
            plus = b"+r%d" % i if k == 4 else b"+"
            if k == 5:
                s, q = s[:40], q[:40]
            if i == 10:
                s, q = (s * 16)[:1400], (q * 16)[:1400]   # past MAX_READ_LENGTH (1210): cut
            if k == 6:
                s, q = s + b"\r", q + b"\r"
            sep = b"\n\n" if k == 7 else b"\n"
            f.write(b"@" + name + sep + s + b"\n" + plus + sep + q + b"\n")
            if k == 8:
                f.write(b"\n")
    pre = cache.get(c.index_key)
    so, do = str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")
    dropin.run(c.meta["program"], "dump", pre, fq, None, so, 2, trim)
    dropin.run(c.meta["program"], "oracle-dropin", pre, fq, None, do, 2, trim)
    a, b = dropin.outputs(so), dropin.outputs(do)
    assert sorted(a) == sorted(b)
    for suf in a:
        assert a[suf] == b[suf], "output %r differs" % (suf or ".sam")
    # (CR bytes stay inside the records: split on LF only)
    recs = [l for l in a[""].split(b"\n") if l and not l.startswith(b"@")]
    assert len(recs) == len(c.r1)
    assert sum(1 for l in recs if not int(l.split(b"\t")[1]) & 4) > 0


def test_oracle_dropin_fastq_bulk_read_matches_stock(cache, tmp_path):
    """The binding's bulk FASTQ reading (a 4 MB buffer refilled by fread, memchr line ends, the FILE
    put back where the character-wise parse would leave it): 30k reads, about 7 MB, so records
    straddle buffer refills; some quality lines end in a 0xFF byte (the reference's `char` compare
    with EOF ends the line there); reads of many lengths -- the stock SAM byte for byte."""
    from tests import dropin
    c = Case("pe_gapped_errmut")
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    fq = str(tmp_path / "r.fq")
    n0 = len(c.r1)
    with open(fq, "wb") as f:
        for i in range(30000):
            s = c.r1.read(i % n0)
            L = 30 + (i * 37) % (len(s) - 29) if i % 5 == 0 else len(s)
            s = s[:L]
            q = bytes(33 + (i * 3 + k * 7) % 41 for k in range(len(s)))
            if i % 11 == 0:
                q = q[:-1] + b"\xff"
            f.write(b"@q%d desc %d\n" % (i, i) + s + b"\n+\n" + q + b"\n")
    pre = cache.get(c.index_key)
    so, do = str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")
    dropin.run(c.meta["program"], "dump", pre, fq, None, so, 2)
    dropin.run(c.meta["program"], "oracle-dropin", pre, fq, None, do, 2)
    a, b = dropin.outputs(so), dropin.outputs(do)
    assert sorted(a) == sorted(b)
    for suf in a:
        assert a[suf] == b[suf], "output %r differs" % (suf or ".sam")
    recs = [l for l in a[""].split(b"\n") if l and not l.startswith(b"@")]
    assert len(recs) == 30000


@pytest.mark.parametrize("kind", ["se", "sj"])
def test_oracle_dropin_remove_neighbour_matches_stock(kind, tmp_path):
    """The binding's anti-supporting read scan and remove_neighbour (the library's decisions, the
    removals mirrored into the reference's site lists) on the two data sets where remove_neighbour
    removes events (tests/golden/make_removed.py): subread-align on 2%-indel reads over a 150 kb
    genome, subjunc on spliced reads over a genome with repeat families.  Event tables before and
    after remove_neighbour (the reference's own dump hook), SAM, VCF and BED identical to stock."""
    from tests import dropin
    from subread_amd import build_index
    from subread_amd.abi import PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import random_genome, simulate_reads, simulate_spliced_reads
    prog = PROGRAM_ALIGN if kind == "se" else PROGRAM_SUBJUNC
    if not have(prog, "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    if kind == "se":
        g = random_genome([150_000], 78)
        reads = simulate_reads(g, 120_000, 100, seed=4, sub=0.005, indel=0.02)
    else:
        g = random_genome([1_000_000, 700_000], 77, repeats=(200, 300, 20, 0.02))
        reads = simulate_spliced_reads(g, 30000, 100, seed=6, spliced=0.5, max_intron=3000)
    fa, pre = str(tmp_path / "g.fa"), str(tmp_path / "idx")
    g.write_fasta(fa)
    build_index(fa, pre, gap=1, force_one_block=True)
    fq = str(tmp_path / "r.fq")
    dropin.write_fastq(fq, reads)
    so, do = str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")
    dropin.run(prog, "dump", pre, fq, None, so, 1, env={"SVG_REF_EVENTS_RN": so + ".rn"})
    dropin.run(prog, "oracle-dropin", pre, fq, None, do, 1, env={"SVG_REF_EVENTS_RN": do + ".rn"})
    rn = np.fromfile(so + ".rn", np.uint8)[8:]
    assert (rn == 0).sum() > 0   # remove_neighbour removed events here
    rep = dropin.compare(so, do)
    assert ".rn" in rep["files"] and rep["mapped"] > 0


@pytest.mark.parametrize("extra,threads", [
    (("--multiMapping", "-B", "3"), 4),           # multi-mapping reads: up to 3 locations, HI / NH, MAPQ
    # no records for unmapped fragments; RG tag (-T 1: the stock aligner hangs at -T > 1 with
    # --ignoreUnmapped: add_buffered_fragment waits for a fragment that is never written, core.c:2435)
    (("--ignoreUnmapped", "--rg-id", "grp1", "--rg", "SM:x"), 1),
    (("-d", "150", "-D", "400", "--noTLENpreference"), 1),
    (("-M", "1", "--complexIndels"), 1),            # mismatch limit, realignment variant distance 1
    (("-P", "6",), 1),                               # Phred+64 qualities: converted in the SAM
])
def test_oracle_dropin_realign_options(extra, threads, cache, tmp_path):
    """iteration two's options through the library's realignment: stock vs drop-in, same bytes."""
    from tests import dropin
    c = Case("pe_gapped_errmut")
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    f1, f2 = dropin.fastq_pair(str(tmp_path), c.name, c.r1, c.r2)
    if "-P" in extra:   # the same reads with Phred+64 qualities
        for f in (f1, f2):
            lines = open(f, "rb").read().split(b"\n")
            for i in range(3, len(lines), 4):
                lines[i] = bytes(min(b + 31, 126) for b in lines[i])
            open(f, "wb").write(b"\n".join(lines))
    pre = cache.get(c.index_key)
    so, do = str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")
    dropin.run(c.meta["program"], "dump", pre, f1, f2, so, threads, extra)
    dropin.run(c.meta["program"], "oracle-dropin", pre, f1, f2, do, threads, extra)
    rep = dropin.compare(so, do)
    assert rep["mapped"] > 0


def _bam_records(path):
    """The alignment records of a BAM file (BGZF members concatenated, header text and reference
    list skipped: the header's @PG line holds the program path)."""
    import gzip
    import struct
    b = gzip.open(path, "rb").read()
    assert b[:4] == b"BAM\x01"
    lt = struct.unpack("<i", b[4:8])[0]
    p = 8 + lt
    nref = struct.unpack("<i", b[p:p + 4])[0]
    p += 4
    for _ in range(nref):
        ln = struct.unpack("<i", b[p:p + 4])[0]
        p += 4 + ln + 4
    return b[p:]


def _bgzf_blocks(path):
    """The BGZF blocks of a BAM file, raw, with their inflated contents: [(raw, data)]."""
    import struct
    import zlib
    b = open(path, "rb").read()
    out, p = [], 0
    while p < len(b):
        assert b[p:p + 4] == b"\x1f\x8b\x08\x04", "not a BGZF block at %d" % p
        bsize = struct.unpack("<H", b[p + 16:p + 18])[0] + 1
        raw = b[p:p + bsize]
        out.append((raw, zlib.decompress(raw[18:-8], -15)))
        p += bsize
    return out


def _bam_blocks_after_header(path):
    """The raw BGZF blocks that follow the header's (the @PG line in the header holds the program
    path, so the header blocks differ between the two programs; the record blocks must not)."""
    import struct
    blocks = _bgzf_blocks(path)
    head = b"".join(d for _, d in blocks)
    lt = struct.unpack("<i", head[4:8])[0]
    p = 8 + lt
    nref = struct.unpack("<i", head[p:p + 4])[0]
    p += 4
    for _ in range(nref):
        ln = struct.unpack("<i", head[p:p + 4])[0]
        p += 4 + ln + 4
    k, got = 0, 0
    while got < p:
        got += len(blocks[k][1])
        k += 1
    assert got == p, "the records share a block with the header"
    return [raw for raw, _ in blocks[k:]]


def _bam_record_list(path):
    """The alignment records of a BAM file, one bytes object each (block_size included)."""
    import struct
    b = _bam_records(path)
    out, p = [], 0
    while p < len(b):
        n = struct.unpack("<i", b[p:p + 4])[0]
        out.append(b[p:p + 4 + n])
        p += 4 + n
    return out


def _mask_nul_tails(ours, theirs):
    """Reads holding NUL bytes (the se_gapped_mixed case): SamBam_read2bin encodes a read's bases up
    to the NUL (sambam-file.c:1460-1476) in a field of l_seq / 2 bytes; the rest of the reference's
    field is whatever its stream buffer held there, ours is zero.  Both records get that part
    masked (it starts at the first all-zero byte of our field)."""
    import struct
    a, b = bytearray(ours), bytearray(theirs)
    name_len, ncig = a[12], struct.unpack("<H", a[16:18])[0]
    l_seq = struct.unpack("<i", a[20:24])[0]
    s0 = 36 + name_len + 4 * ncig
    s1 = s0 + (l_seq + 1) // 2
    z = a.find(b"\x00", s0, s1)
    if z >= 0:
        a[z:s1] = bytes(s1 - z)
        b[z:s1] = bytes(s1 - z)
    return bytes(a), bytes(b)


@pytest.mark.parametrize("name,threads,keep,chunk", [
    ("pe_gapped_errmut", 4, True, 0),        # --keepReadOrder at -T 4: the reference's ordered stream (writer id -1 / -2)
    ("pe_gapped_errmut", 1, False, 0),       # -T 1: the same ordered stream (write_single_fragment, core.c:2144-2151)
    ("pe_gapped_errmut", 1, False, 600),     # four read chunks: an open block crosses each chunk boundary
    ("sj_pe_gapped_long", 1, False, 0),      # subjunc PE > 160 bp: XS tags, long records
    ("se_gapped_mixed_n14_I16", 4, True, 0), # single end: every record closes a location
    ("pe_gapped_errmut", 4, False, 0),       # the default: the reference's threads write unordered blocks
])
def test_oracle_dropin_bam_matches_stock(name, threads, keep, chunk, cache, tmp_path):
    """BAM output (the reference's default, no --SAMoutput) through the library's iteration two and
    its BAM sink (svg_sam_writer_open_bam, svg_bam_format): with the reference's ordered stream
    (-T 1, --keepReadOrder) every record block after the header is byte-identical to the stock
    aligner's -- the same records, cut into the same BGZF blocks, deflated the same way; without
    --keepReadOrder the stock aligner's threads write their blocks in whatever order they finish, and
    the records are the same multiset.  VCF / BED identical, every stage the library's."""
    from tests import dropin
    c = Case(name)
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    f1, f2 = dropin.fastq_pair(str(tmp_path), c.name, c.r1, c.r2)
    pre = cache.get(c.index_key)
    extra = dropin.case_extra(c) + (["--keepReadOrder"] if keep else [])
    env = {"SVG_REF_READS_PER_CHUNK": str(chunk)} if chunk else None
    so, do = str(tmp_path / "stock.bam"), str(tmp_path / "dropin.bam")
    dropin.run(c.meta["program"], "dump", pre, f1, f2, so, threads, extra, env=env, sam=False)
    r = dropin.run(c.meta["program"], "oracle-dropin", pre, f1, f2, do, threads, extra, env=env, sam=False)
    st = dropin.assert_library(r.stderr)
    if chunk:
        assert st["iteration_two"][0] >= 4
    a, b = _bam_record_list(so), _bam_record_list(do)
    assert len(a) == len(c.r1) * c.ends
    if "mixed" in name:   # reads with NUL bytes: compare outside the stale part of their 4-bit field
        pairs = [_mask_nul_tails(y, x) for x, y in zip(a, b)]
        assert sum(x != y for x, y in zip(a, b)) < len(a) // 10
        a, b = [t for _, t in pairs], [o for o, _ in pairs]
    if threads == 1 or keep:
        assert a == b
        if "mixed" not in name:
            assert _bam_blocks_after_header(so) == _bam_blocks_after_header(do)
    else:
        assert sorted(a) == sorted(b)
    for suf in (".indel.vcf", ".junction.bed"):
        if os.path.exists(so + suf):
            assert open(so + suf, "rb").read() == open(do + suf, "rb").read(), suf


@pytest.mark.parametrize("name,threads,chunk", [
    ("pe_gapped_errmut", 1, 500),          # one thread: every chunk adds to the global event table (its sorted site lists)
    ("pe_gapped_errmut", 4, 500),          # per-thread tables merged into the global one, chunk after chunk
    ("sj_pe_mb_long_gappedM6", 1, 150),    # 4-block index, long subjunc pairs: windows per block, tables across chunks
    ("se_gapped_mixed_n14_I16", 2, 700),   # -n 14 -I 16, N / IUPAC
])
def test_oracle_dropin_several_chunks(name, threads, chunk, cache, tmp_path):
    """Inputs run as several read chunks (SVG_REF_READS_PER_CHUNK, both programs): the event table,
    its site lists, the expected-TLEN estimate and the SAM stream cross chunk boundaries as in a run
    of more than 6.7M reads -- the stock outputs byte for byte, every stage the library's."""
    c = Case(name)
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "oracle-dropin", threads,
                     env={"SVG_REF_READS_PER_CHUNK": str(chunk)}, stock_env={"SVG_REF_READS_PER_CHUNK": str(chunk)})
    assert rep["stages"]["iteration_two"][0] >= 3 and rep["mapped"] > 0


@pytest.mark.parametrize("name,threads", [("pe_gapped_errmut", 4), ("sj_pe_gapped_junc", 1)])   # (the stock subjunc's event dump at -T > 1 varies run to run)
def test_oracle_dropin_third_iteration(name, threads, cache, tmp_path):
    """-I 20 (> 16: the reference's third iteration, do_iteration_three, core.c:3643-3647, reads the
    records and flags iteration two leaves): the stock outputs incl. the reassembly FASTA."""
    from tests import dropin
    c = Case(name)
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    f1, f2 = dropin.fastq_pair(str(tmp_path), c.name, c.r1, c.r2)
    pre = cache.get(c.index_key)
    so, do = str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")
    dropin.run(c.meta["program"], "dump", pre, f1, f2, so, threads, ["-I", "20"])
    r = dropin.run(c.meta["program"], "oracle-dropin", pre, f1, f2, do, threads, ["-I", "20"])
    dropin.assert_library(r.stderr)
    rep = dropin.compare(so, do)
    assert ".reassembly.fa" in rep["files"] or c.meta["program"] == 1


@pytest.mark.parametrize("env,stage", [({"SVG_REF_ITER2": "1"}, "iteration_two"), ({"SVG_REF_EVENTSTAGE": "1"}, "events"),
                                        ({"SVG_REF_ANTI": "1"}, "anti_support")])
def test_oracle_dropin_fallbacks_are_counted(env, stage, cache, tmp_path):
    """A stage forced onto the reference's own function: the outputs stay the stock program's (by
    construction), the stage counter says "reference", and SVG_REQUIRE_LIBRARY=1 turns the same run
    into an error (exit status 3, the stage and the reason on stderr) -- a fallback never passes as
    the library's work."""
    import subprocess
    from tests import dropin
    c = Case("pe_gapped_errmut")
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    f1, f2 = dropin.fastq_pair(str(tmp_path), c.name, c.r1, c.r2)
    pre = cache.get(c.index_key)
    so, do = str(tmp_path / "stock.sam"), str(tmp_path / "dropin.sam")
    dropin.run(c.meta["program"], "dump", pre, f1, f2, so, 2)
    r = dropin.run(c.meta["program"], "oracle-dropin", pre, f1, f2, do, 2, env=dict(env, SVG_REQUIRE_LIBRARY="0"))
    st = dropin.stages(r.stderr)
    assert st[stage][1] > 0 and st[stage][0] == 0, st
    assert st["vote"][1] == 0 and st["vote"][0] > 0
    dropin.compare(so, do)
    args = [dropin.binary(0, "oracle-dropin"), "-T", "2", "-i", pre, "-r", f1, "-R", f2, "-o", str(tmp_path / "x.sam"),
            "--SAMoutput", "-t", "1"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=900, env=dict(os.environ, SVG_REQUIRE_LIBRARY="1", **env))
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "SVG_REQUIRE_LIBRARY=1: stage %s fell back" % stage in r.stderr


@pytest.mark.parametrize("name,threads", [("pe_gapped_errmut", 1), ("sj_pe_gapped_long", 1), ("sj_pe_mb_long_gappedM6", 1),
                                          ("se_gapped_mixed_n14_I16", 4)])
def test_oracle_dropin_several_handles(name, threads, cache, tmp_path):
    """SVG_DEVICES=0,0,0: the binding with three handles (svg_attach_devices) splits each chunk into
    three contiguous read ranges voted by three host threads into the one bigtable (the GPU fan-out
    of run_maybe_threads, core.c:3379-3461) -- the stock reference's outputs byte for byte, incl.
    the multi-block loop and fragile junction voting (on the first handle)."""
    c = Case(name)
    if not have(c.meta["program"], "oracle-dropin"):
        pytest.skip("reference drop-in binaries not built (make -C oracle dropin)")
    rep = check_case(c, cache.get(c.index_key), str(tmp_path), "oracle-dropin", threads, env={"SVG_DEVICES": "0,0,0"})
    assert rep["mapped"] > 0
