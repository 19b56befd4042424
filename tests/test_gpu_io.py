"""GPU: the host-buffer pipeline and the packed read form, through the C ABI.

* svg_vote_batch_packed (2-bit reads, back to back or fixed stride, with and without
  the exception mask) gives the reference's golden records byte for byte;
* the compacted download (only non-zero records cross PCIe, expanded on the host by
  worker threads) is exact for many small sub-batches and thread counts, SE/PE/subjunc;
* svg_vote_batch_packed_device (packed reads in HBM);
* the read-length bound of the device entry points is enforced (svg_device_status), and
  calls given different streams are ordered on the handle's shared buffers."""
import numpy as np
import pytest

from tests.common import Case, golden_names, ensure_built, pack_records, describe_mismatch

ensure_built()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_indexes(index_cache):
    import subread_amd as sa
    cache = {}

    def get(key):
        if key not in cache:
            cache[key] = sa.VoteIndex(index_cache.get(key), device=0)
        return cache[key]
    yield get
    for v in cache.values():
        v.close()


@pytest.mark.parametrize("layout", ["packed", "stride"])
@pytest.mark.parametrize("name", golden_names())
def test_packed_matches_reference_golden(name, layout, gpu_indexes):
    import subread_amd as sa
    c = Case(name)
    ix = gpu_indexes(c.index_key)
    stride = None
    if layout == "stride":
        stride = int(max(c.r1.lens.max(), c.r2.lens.max() if c.r2 is not None else 0))
    p1 = sa.pack_reads(c.r1, stride)
    p2 = sa.pack_reads(c.r2, stride) if c.r2 is not None else None
    out, jout, bm = ix.vote_packed(c.params, p1, p2)
    got = pack_records(out, jout, bm)
    assert (got == c.expected).all(), describe_mismatch(got, c.expected, c.ends, c.params.multi_best)


def test_packed_mask_is_exercised():
    import subread_amd as sa
    assert sa.pack_reads(Case("se_full_mixed").r1, None).xmask is not None


@pytest.mark.parametrize("mode", ["se", "pe", "sj"])
@pytest.mark.parametrize("entry", ["ascii", "packed"])
def test_compacted_pipeline_small_subbatches(mode, entry, gpu_indexes, index_cache, svgopt):
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_ALIGN, PROGRAM_SUBJUNC
    from subread_amd.sim import Genome, simulate_reads, simulate_spliced_reads
    key = "chr901_full"
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta("chr901"))
    n = 20011
    if mode == "sj":
        r1, r2 = simulate_spliced_reads(g, n, 100, seed=41), None
    else:
        r1 = simulate_reads(g, n, 100, seed=42, sub=0.02, indel=0.02, nrate=0.002)
        r2 = simulate_reads(g, n, 100, seed=43, sub=0.02, indel=0.02) if mode == "pe" else None
    p = default_params(PROGRAM_SUBJUNC if mode == "sj" else PROGRAM_ALIGN, mode == "pe")
    ref, rj, rbm, _ = OracleIndex(pre).vote(p, r1, r2, threads=16)
    want = pack_records(ref, rj if mode == "sj" else None, rbm if mode == "sj" else None)
    ix = gpu_indexes(key)
    # (2000 and 64: the ramped schedule -- sub/4, sub/2, full ones, the remainder, sub/2, sub/4;
    # 3001 / 7777 and host_ramp 0: uniform sub-batches)
    for sub, th, ramp in (("3001", "1", 1), ("7777", "3", 1), ("64", "8", 1), ("2000", "4", 1), ("2000", "2", 0)):
        svgopt.set("host_sub", int(sub))
        svgopt.set("host_threads", int(th))
        svgopt.set("host_ramp", ramp)
        if entry == "ascii":
            out, jout, bm = ix.vote(p, r1, r2)
        else:
            out, jout, bm = ix.vote_packed(p, sa.pack_reads(r1, 100), sa.pack_reads(r2, None) if r2 is not None else None)
        got = pack_records(out, jout if mode == "sj" else None, bm if mode == "sj" else None)
        assert (got == want).all(), "sub %s: %s" % (sub, describe_mismatch(got, want, 2 if mode == "pe" else 1, 3))


@pytest.mark.parametrize("name", ["se_mb_long_gappedM6", "sj_pe_mb_long_gappedM6", "pe_mb_long_fullM17"])
@pytest.mark.parametrize("entry", ["ascii", "packed"])
def test_compacted_pipeline_multi_block(name, entry, gpu_indexes, index_cache, svgopt):
    """Multi-block indexes through the host pipeline with many sub-batches: later blocks run on
    the first block's stream from the stored records of each sub-batch, device and staging slots
    are reused; golden records (4-6 blocks) and the oracle on 15k simulated reads of the genome."""
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    from subread_amd.sim import Genome, simulate_pairs, simulate_spliced_reads, simulate_reads
    c = Case(name)
    ix = gpu_indexes(c.index_key)
    assert ix.n_blocks > 1
    for sub, th in (("97", "2"), ("1000", "5")):
        svgopt.set("host_sub", int(sub))
        svgopt.set("host_threads", int(th))
        if entry == "ascii":
            out, jout, bm = ix.vote(c.params, c.r1, c.r2)
        else:
            out, jout, bm = ix.vote_packed(c.params, sa.pack_reads(c.r1, None),
                                           sa.pack_reads(c.r2, None) if c.r2 is not None else None)
        got = pack_records(out, jout, bm)
        assert (got == c.expected).all(), "sub %s: %s" % (sub, describe_mismatch(got, c.expected, c.ends, 3))
    g = Genome.read_fasta(index_cache.genome_fasta(c.index_key.rsplit("_", 1)[0]))
    n = 15013
    if c.params.do_breakpoint_detection:
        r1, r2 = simulate_spliced_reads(g, n, 150, seed=61, max_intron=20000), None
        if c.r2 is not None:
            r2 = simulate_spliced_reads(g, n, 150, seed=62, max_intron=20000)
    elif c.r2 is not None:
        r1, r2 = simulate_pairs(g, n, 150, seed=63, sub=0.01)
    else:
        r1, r2 = simulate_reads(g, n, 100, seed=64, sub=0.02, indel=0.02, nrate=0.002), None
    ref, rj, rbm, _ = OracleIndex(index_cache.get(c.index_key)).vote(c.params, r1, r2, threads=16)
    sj = bool(c.params.do_breakpoint_detection)
    want = pack_records(ref, rj if sj else None, rbm if sj else None)
    svgopt.set("host_sub", 3001)
    svgopt.set("host_threads", 3)
    if entry == "ascii":
        out, jout, bm = ix.vote(c.params, r1, r2)
    else:
        out, jout, bm = ix.vote_packed(c.params, sa.pack_reads(r1, None), sa.pack_reads(r2, None) if r2 is not None else None)
    got = pack_records(out, jout if sj else None, bm if sj else None)
    assert (got == want).all(), describe_mismatch(got, want, c.ends, 3)


def _to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)


@pytest.mark.parametrize("chunking", ["default", "ramped", "flat"])
def test_packed_device_entry(chunking, gpu_indexes, svgopt):
    """svg_vote_batch_packed_device on the golden pairs, with the default chunk (one chunk) and
    with small chunks on the two-stream chunk pipeline -- ramped at both ends (chunk/4, chunk/2
    first and last) or uniform (host_ramp 0)."""
    import torch
    import subread_amd as sa
    from subread_amd.abi import SvgPackedReads
    c = Case("pe_full_errmut")
    ix = gpu_indexes(c.index_key)
    dev = torch.device("cuda", 0)
    keep = []

    def dq(pb):
        t = [_to_dev(pb.bases, dev), _to_dev(pb.lens, dev)]
        q = SvgPackedReads()
        q.bases, q.lens = t[0].data_ptr(), t[1].data_ptr()
        q.xmask = None
        if pb.xmask is not None:
            t.append(_to_dev(pb.xmask, dev))
            q.xmask = t[-1].data_ptr()
        q.starts = None
        if pb.starts is not None:
            t.append(_to_dev(pb.starts, dev))
            q.starts = t[-1].data_ptr()
        q.stride, q.n_reads = pb.stride, len(pb)
        keep.append(t)
        return q
    n, mb = len(c.r1), c.params.multi_best
    if chunking != "default":
        assert n >= 8 * 97
        svgopt.set("chunk", 97)
        svgopt.set("overlap", 1)
        svgopt.set("host_ramp", 1 if chunking == "ramped" else 0)
    ix.set_max_read_length(int(max(c.r1.lens.max(), c.r2.lens.max())))
    for stride in (None, 100):
        d_out = torch.zeros(n * 2 * mb * 68, dtype=torch.uint8, device=dev)
        ix.vote_packed_device(c.params, dq(sa.pack_reads(c.r1, stride)), dq(sa.pack_reads(c.r2, stride)),
                              d_out.data_ptr())
        ix.device_status()
        got = d_out.cpu().numpy().reshape(n, -1)
        assert (got == c.expected).all(), describe_mismatch(got, c.expected, 2, mb)
    ix.set_max_read_length(256)


def test_device_read_length_bound_is_enforced(gpu_indexes, index_cache):
    import torch
    import subread_amd as sa
    from subread_amd.abi import default_params
    from subread_amd.sim import Genome, simulate_reads
    ix = gpu_indexes("chr901_full")
    g = Genome.read_fasta(index_cache.genome_fasta("chr901"))
    r = simulate_reads(g, 3000, 250, seed=3)
    dev = torch.device("cuda", 0)
    seq, off, ln = _to_dev(r.seq, dev), _to_dev(r.offsets, dev), _to_dev(r.lens, dev)
    d_out = torch.zeros(len(r) * 3 * 68, dtype=torch.uint8, device=dev)
    p = default_params()
    ix.set_max_read_length(150)
    try:
        ix.vote_device(p, (seq.data_ptr(), off.data_ptr(), ln.data_ptr(), len(r)), None, d_out.data_ptr())
        with pytest.raises(sa.SvgError):
            ix.device_status()
        assert (d_out.cpu().numpy() == 0).all()     # offending reads get zero records
        ix.device_status()                          # the error was cleared
    finally:
        ix.set_max_read_length(256)
    # the host entry point measures its own batch: no error, real records
    out, _, _ = ix.vote(p, r)
    assert (out["selected_votes"][:, 0, 0] > 0).mean() > 0.9


def test_calls_on_different_streams_are_ordered(gpu_indexes):
    import torch
    a, b = Case("se_full_errmut"), Case("se_full_mixed")
    assert a.index_key == b.index_key
    ix = gpu_indexes(a.index_key)
    dev = torch.device("cuda", 0)
    outs = []
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    plan = ((a, streams[0]), (b, streams[1]), (a, streams[1]), (b, streams[0]))
    for c, s in plan:
        d = (_to_dev(c.r1.seq, dev), _to_dev(c.r1.offsets, dev), _to_dev(c.r1.lens, dev))
        outs.append((c, torch.zeros(len(c.r1) * 3 * 68, dtype=torch.uint8, device=dev), d))
    torch.cuda.synchronize()
    # four calls back to back, alternating streams, no host synchronisation in between
    for (c, o, d), (_, s) in zip(outs, plan):
        ix.vote_device(c.params, (d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(c.r1)), None, o.data_ptr(),
                       stream=s.cuda_stream)
    ix.device_status()
    torch.cuda.synchronize()
    for c, o, _ in outs:
        got = o.cpu().numpy().reshape(len(c.r1), -1)
        assert (got == c.expected).all(), describe_mismatch(got, c.expected, 1, 3)


def test_handles_share_the_device_stream_set(index_cache):
    """Every handle on a device uses the device's one set of library streams (svg_vote.hip
    streams_acquire: four streams created back to back, so the chunk pipeline's two kernel
    streams sit on different hardware queues however many indexes a process holds).  Three
    handles of two indexes, host-path calls interleaved without synchronisation, handles closed
    in between (the set lives while any handle does, and is made again after the last close):
    every call gives the reference's golden records."""
    import subread_amd as sa
    a, b = Case("se_full_errmut"), Case("pe_gapped_errmut")
    for rnd in range(2):
        h1 = sa.VoteIndex(index_cache.get(a.index_key), device=0)
        h2 = sa.VoteIndex(index_cache.get(b.index_key), device=0)
        h3 = sa.VoteIndex(index_cache.get(a.index_key), device=0)
        try:
            for k, (h, c) in enumerate(((h1, a), (h2, b), (h3, a), (h2, b), (h1, a))):
                out, _, _ = h.vote(c.params, c.r1, c.r2)
                got = pack_records(out, None, None)
                assert (got == c.expected).all(), "round %d call %d: %s" % (rnd, k, describe_mismatch(got, c.expected, c.ends, 3))
                if k == 2:
                    h3.close()
                    h3 = None
        finally:
            for h in (h1, h2, h3):
                if h is not None:
                    h.close()
