"""GPU: fragile junction voting of subjunc reads > 160 bp (svg_fragile_batch, svg_fragile.hip;
core_fragile_junction_voting, core-junction.c:5151-5422) -- every window record (junction
split and sides, GT/AG strand) and every reported top-vote slot (position, indel recorder)
byte-identical to the CPU restatement (oracle/svoracle.c svo_fragile_batch), whose events are
pinned to the reference's own event tables in tests/test_events.py:
  * the golden long subjunc cases (full, gapped and 4-block indexes, SE and PE);
  * simulated spliced reads of 161-1209 bases on full / gapped / multi-block indexes, SE and PE,
    with mismatches, indels and N bases.
The reference-event check of the GPU windows themselves is test_events.py's GPU test."""
import numpy as np
import pytest

from tests.common import Case, ensure_built

ensure_built()
pytestmark = pytest.mark.gpu

LONG_CASES = ["sj_se_full_long", "sj_pe_gapped_long", "sj_se_mb_synth_long_fullM1"]


def _same(got, want):
    (gw, gs), (ww, ws) = got, want
    assert len(gw) == len(ww), (len(gw), len(ww))
    bad = np.nonzero(gw.view(np.uint8).reshape(len(gw), -1) != ww.view(np.uint8).reshape(len(ww), -1))[0]
    assert not len(bad), "%d windows differ, first: gpu %s / cpu %s" % (len(set(bad)), gw[bad[0]], ww[bad[0]])
    assert len(gs) == len(ws), (len(gs), len(ws))
    assert (gs.view(np.uint8) == ws.view(np.uint8)).all(), "reported slots differ"


@pytest.mark.parametrize("name", LONG_CASES)
def test_fragile_windows_golden_cases(name, index_cache):
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    c = Case(name)
    pre = index_cache.get(c.index_key)
    ix = sa.VoteIndex(pre, device=0)
    got = ix.fragile(c.params, c.r1, c.r2)
    ix.close()
    want = OracleIndex(pre).fragile(c.params, c.r1, c.r2)
    _same(got, want)
    assert got[0]["junction"].sum() > 0


def _spliced(g, n, lens, seed):
    from subread_amd.abi import ReadBatch
    from subread_amd.sim import simulate_spliced_reads
    parts = [simulate_spliced_reads(g, n, L, seed=seed + L, max_intron=20000) for L in lens]
    reads = [b.read(i) for b in parts for i in range(len(b))]
    rng = np.random.default_rng(seed)
    out = []
    for r in reads:   # sprinkle N and a few 1-3 base indels
        r = bytearray(r)
        if rng.random() < 0.2:
            at = int(rng.integers(20, len(r) - 20))
            if rng.random() < 0.5:
                del r[at:at + int(rng.integers(1, 4))]
            else:
                r[at:at] = bytes(rng.choice(list(b"ACGT"), int(rng.integers(1, 4))))
        for i in rng.choice(len(r), int(rng.integers(0, 3)), replace=False):
            r[int(i)] = ord("N")
        out.append(bytes(r))
    return ReadBatch.from_list(out)


@pytest.mark.parametrize("probe", ["image", "literal"])
@pytest.mark.parametrize("key,paired", [("chr901_full", False), ("chr901_gapped", True), ("long777_gappedM6", False),
                                        ("synth4242_fullM1", True)])
def test_fragile_windows_simulated(key, paired, probe, index_cache, svgopt):
    """probe: the equal-key runs from the probe images (bucket code / key-hash, go_run) or the literal
    gehash_go_q search (option keys_literal) -- identical windows either way"""
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    from subread_amd.abi import default_params, PROGRAM_SUBJUNC
    from subread_amd.sim import Genome
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta(key.rsplit("_", 1)[0]))
    lens = (161, 200, 257, 400, 700, 1209)
    r1 = _spliced(g, 150, lens, 71)
    r2 = _spliced(g, 150, lens, 83) if paired else None
    p = default_params(PROGRAM_SUBJUNC, paired)
    svgopt.set("keys_literal", 1 if probe == "literal" else 0)
    ix = sa.VoteIndex(pre, device=0)
    got = ix.fragile(p, r1, r2)
    ix.close()
    want = OracleIndex(pre).fragile(p, r1, r2)
    _same(got, want)
    assert want[0]["junction"].sum() > 0
