"""Host post-vote events (include/subread_events.h): the indel / junction event table the
reference builds from the vote records in its final voting run (find_new_indels,
core-indel.c:1831; find_new_junctions, core-junction.c:3836; merged by
finalise_indel_and_junction_thread, core-indel.c:1012) and the CORE_IS_GAPPED_READ marks on
the records.  Known answers: tests/golden/events/<case>.npz, dumped from the reference run
with -T 1 (tests/golden/make_golden.py, oracle/ref_dump_hook.c).

CPU tests feed the reference's own records (the golden vote dump); the GPU test feeds the
records of the HIP vote path."""
import glob
import os

import numpy as np
import pytest

from subread_amd.abi import EVENT_DTYPE, MAPPING_DTYPE, SUBJUNC_DTYPE, BIG_MARGIN_WORDS
from tests.common import GOLD, Case, ensure_built

ensure_built()

EVENT_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "events", "*.npz")))


def load_events(name):
    z = np.load(os.path.join(GOLD, "events", name + ".npz"), allow_pickle=False)
    return z["events"].copy().view(EVENT_DTYPE).reshape(-1), z["flags"]


def split_records(c):
    """golden vote dump -> (mapping, subjunc|None, big_margin|None) arrays"""
    n, mb, e = len(c.r1), c.params.multi_best, c.ends
    raw = c.expected
    out = raw[:, :e * mb * 68].copy().view(MAPPING_DTYPE).reshape(n, e, mb)
    o, jout, bm = e * mb * 68, None, None
    if c.params.do_breakpoint_detection:
        jout = raw[:, o:o + e * mb * 16].copy().view(SUBJUNC_DTYPE).reshape(n, e, mb)
        o += e * mb * 16
    if c.params.do_big_margin_filtering_for_junctions:
        bm = raw[:, o:o + e * BIG_MARGIN_WORDS * 2].copy().view(np.uint16).reshape(n, e, BIG_MARGIN_WORDS)
    return out, jout, bm


def describe(got, want, limit=4):
    if len(got) != len(want):
        g = set((int(x["small_side"]), int(x["large_side"]), int(x["indel_length"])) for x in got)
        w = set((int(x["small_side"]), int(x["large_side"]), int(x["indel_length"])) for x in want)
        return "%d events, reference %d; only ours %s; only reference %s" % (len(got), len(want), sorted(g - w)[:5],
                                                                           sorted(w - g)[:5])
    bad = np.nonzero((got.view(np.uint8).reshape(len(got), -1) != want.view(np.uint8).reshape(len(want), -1)).any(1))[0]
    return "\n".join(["%d of %d events differ" % (len(bad), len(got))] +
                     ["  ours %s\n  ref  %s" % (got[i], want[i]) for i in bad[:limit]])


def long_subjunc(c):
    return bool(c.params.do_breakpoint_detection) and (
        c.r1.lens.max() > 160 or (c.r2 is not None and c.r2.lens.max() > 160))


def quals_of(batch):
    """the fixtures' FASTQ qualities (tests/golden/make_golden.py writes 'I' for every base)"""
    from subread_amd.abi import ReadBatch
    return ReadBatch(np.full(batch.seq.size, ord("I"), np.uint8), batch.offsets, batch.lens)


def extras(c, windows):
    """quals / fragile arguments of find_events for a case (None for the short-read cases)"""
    if not long_subjunc(c):
        return {}
    return dict(quals=(quals_of(c.r1), quals_of(c.r2) if c.r2 is not None else None), fragile=windows)


def check(got, flags, want, wflags):
    assert len(got) == len(want) and (got.view(np.uint8) == want.view(np.uint8)).all(), describe(got, want)
    assert (flags == wflags).all(), "%d records' flags differ" % int((flags != wflags).sum())


@pytest.mark.parametrize("name", EVENT_CASES)
def test_events_match_reference(name, index_cache):
    """The reference's records -> our event stage; for subjunc reads > 160 bp the fragile
    junction voting windows come from the CPU restatement (the GPU's are checked against it in
    tests/test_gpu_fragile.py)."""
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    c = Case(name)
    want, wflags = load_events(name)
    pre = index_cache.get(c.index_key)
    g = sa.GenomeArrays(pre)
    recs = split_records(c)
    windows = OracleIndex(pre).fragile(c.params, c.r1, c.r2) if long_subjunc(c) else None
    got = sa.find_events(g, c.params, c.r1, c.r2, recs, **extras(c, windows))
    check(got, recs[0]["result_flags"].reshape(-1).view(np.uint16), want, wflags)
    g.close()


def test_events_merge_of_shards_equals_one_table(index_cache):
    """Per-shard tables merged like the reference's per-thread tables give the same support
    counts and event set as one table over all reads (critical_read_id and inserted bases
    come from the first record of a group, as in one table)."""
    import subread_amd as sa
    c = Case("sj_pe_gapped_junc")
    g = sa.GenomeArrays(index_cache.get(c.index_key))
    whole, _ = load_events(c.name)
    out, jout, bm = split_records(c)
    tables = []
    cuts = [0, 333, 1000, len(c.r1)]
    for a, b in zip(cuts[:-1], cuts[1:]):
        t = sa.EventTable()
        t.add_batch(g, c.params, c.r1.slice(a, b), c.r2.slice(a, b), (out[a:b], jout[a:b], bm[a:b]), first_read=a)
        tables.append(t)
    m = sa.EventTable.merge(tables).events()
    key = ["small_side", "large_side", "indel_length", "supporting_reads", "event_type"]
    assert len(m) == len(whole)
    for k in key:
        assert (m[k] == whole[k]).all(), k
    g.close()


def test_events_need_fragile_windows_for_long_subjunc_reads(index_cache):
    """svg_events_add_batch (no fragile windows) refuses subjunc reads > 160 bp rather than
    leaving out the fragile junction voting's events."""
    import subread_amd as sa
    c = Case("sj_pe_gapped_long")
    g = sa.GenomeArrays(index_cache.get(c.index_key))
    with pytest.raises(sa.SvgError, match="fragile junction votes"):
        sa.find_events(g, c.params, c.r1, c.r2, split_records(c))
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in EVENT_CASES if len(load_events(n)[0]) > 0])
def test_gpu_records_give_reference_events(name, index_cache):
    """The whole drop-in stage: HIP vote -> host events == the reference's event table."""
    import subread_amd as sa
    c = Case(name)
    want, wflags = load_events(name)
    pre = index_cache.get(c.index_key)
    ix = sa.VoteIndex(pre, device=0)
    out, jout, bm = ix.vote(c.params, c.r1, c.r2)
    windows = ix.fragile(c.params, c.r1, c.r2) if long_subjunc(c) else None
    ix.close()
    g = sa.GenomeArrays(pre)
    got = sa.find_events(g, c.params, c.r1, c.r2, (out, jout, bm), **extras(c, windows))
    check(got, out["result_flags"].reshape(-1).view(np.uint16), want, wflags)
    g.close()


RN_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "events_rn", "*.npz")))


@pytest.mark.parametrize("name", [n for n in RN_CASES if not n.startswith("rn_")])
def test_remove_neighbour_after_event_stage_matches_reference(name, index_cache):
    """The event stage, the anti-supporting read scan and remove_neighbour (core-indel.c:447) on
    the reference's records give the reference's event types after remove_neighbour
    (tests/golden/events_rn, made by tests/golden/make_removed.py with the reference itself).
    These cases remove nothing; the rn_* cases below do."""
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    c = Case(name)
    want = np.load(os.path.join(GOLD, "events_rn", name + ".npz"), allow_pickle=False)["types"]
    pre = index_cache.get(c.index_key)
    g = sa.GenomeArrays(pre)
    recs = split_records(c)
    windows = OracleIndex(pre).fragile(c.params, c.r1, c.r2) if long_subjunc(c) else None
    got = sa.find_events(g, c.params, c.r1, c.r2, recs, remove_neighbour=True, **extras(c, windows))
    g.close()
    assert len(got) == len(want) and (got["event_type"] == want).all()


@pytest.mark.parametrize("name", [n for n in RN_CASES if n.startswith("rn_")])
def test_remove_neighbour_matches_reference(name):
    """svg_events_remove_neighbour on the reference's own event table (dumped right before its
    remove_neighbour) removes exactly the events the reference removes: same-length indels
    within 3 bases (rn_se: 41 of 4789) and junctions within 11 bases (rn_sj: 8 of 11999), with
    the reference's quality / support / coordinate tie-breaks."""
    import subread_amd as sa
    z = np.load(os.path.join(GOLD, "events_rn", name + ".npz"), allow_pickle=False)
    before, want = z["events"], z["types"]
    t = sa.EventTable()
    t.load(before)
    t.remove_neighbour()
    got = t.events()
    t.close()
    assert len(got) == len(want)
    removed_ref = np.nonzero(want == 0)[0]
    removed_ours = np.nonzero(got["event_type"] == 0)[0]
    assert len(removed_ref) > 0
    assert (got["event_type"] == want).all(), "removed: ours %s, reference %s" % (
        sorted(set(removed_ours) - set(removed_ref))[:8], sorted(set(removed_ref) - set(removed_ours))[:8])
    # everything else unchanged
    b = before.view(EVENT_DTYPE).reshape(-1)
    keep = want != 0
    assert (got[keep].view(np.uint8) == b[keep].view(np.uint8)).all()


def test_genome_arrays_contigs_are_sam_header_lengths(tmp_path):
    """svg_genome_arrays_contigs gives write_sam_headers' @SQ lengths (FETCH_SEQ_LEN, core.c:3841:
    read_offsets delta + 16 - 2 * padding): the FASTA's contig lengths for an index the reference's
    builder layout pads with 1210 bases, and -- where the stock aligner is built -- its own @SQ lines."""
    import subread_amd as sa
    from subread_amd.sim import random_genome, simulate_reads
    from tests import dropin
    g = random_genome([150_000, 70_001, 33_333, 5_000], 4242)
    fa, pre = str(tmp_path / "g.fa"), str(tmp_path / "idx")
    g.write_fasta(fa)
    sa.build_index(fa, pre)   # (gapped: a small .tab; the contig table is the same for every index kind)
    got = sa.GenomeArrays(pre).contigs()
    assert got == [(n, len(s)) for n, s in zip(g.names, g.seqs)]
    if not dropin.have(0, "dump"):
        return
    fq = str(tmp_path / "r.fq")
    dropin.write_fastq(fq, simulate_reads(g, 50, 100, seed=3))
    out = str(tmp_path / "o.sam")
    dropin.run(0, "dump", pre, fq, None, out)
    sq = [l.split(b"\t") for l in open(out, "rb").read().splitlines() if l.startswith(b"@SQ")]
    assert [(f[1][3:].decode(), int(f[2][3:])) for f in sq] == got
