"""GPU: parity at full size against the reference itself (SURVEY.md §8(c) fixture plan).

All 10M C2 reads (bench.py workload c2) are voted through svg_vote_batch_packed (the metric's
entry point: host buffers, 1M-read sub-batches, compacted download, host expansion) and the
SHA-256 of the n x 3 x 68-byte records is compared with tests/golden/c2_digest.json, which
tests/golden/make_c2_digest.py computed from the reference aligner's own vote dump
(oracle/_ref/subread-align-dump on the same reads and the reference-built index).  Per-1M-read
block digests name the first differing block."""
import hashlib
import json
import os

import numpy as np
import pytest

from tests.common import GOLD

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_c2_10m_records_match_reference_digest():
    import subread_amd as sa
    from subread_amd.abi import default_params
    from subread_amd.sim import random_genome, simulate_reads
    want = json.load(open(os.path.join(GOLD, "c2_digest.json")))
    n = want["n_reads"]
    g = random_genome([1_000_000], 901)
    ix = sa.VoteIndex.build_genome(g, gap=1, force_one_block=True, device=0)
    try:
        rb = simulate_reads(g, n, 100, seed=20261015, first=0, sub=0.01, indel=0.001)
        pk = sa.pack_reads(rb, 100, threads=16)
        out, _, _ = ix.vote_packed(default_params(), pk)
        raw = out.view(np.uint8).reshape(n, -1)
        assert raw.shape[1] == 3 * 68
        B = want["block_reads"]
        got_blocks = [hashlib.sha256(raw[a:a + B].tobytes()).hexdigest() for a in range(0, n, B)]
        bad = [i for i, (a, b) in enumerate(zip(got_blocks, want["block_sha256"])) if a != b]
        assert not bad, "records differ from the reference in 1M-read blocks %s" % bad
        assert hashlib.sha256(raw.tobytes()).hexdigest() == want["sha256"]
        assert int((out["selected_votes"][:, 0, 0] > 0).sum()) == want["reads_with_votes"]
    finally:
        ix.close()


@pytest.mark.timeout(900)
def test_c3_50m_records_match_reference_digest():
    """The bench workload itself: all 50M C3 reads (3.0 Gbp genome with repeat families, full
    index built in HBM) through svg_vote_batch_packed, against tests/golden/c3_digest.json --
    the SHA-256 of the reference aligner's own post-vote records of the same reads
    (tools/c3_reference_digest.py)."""
    import subread_amd as sa
    from subread_amd.abi import default_params
    from subread_amd.sim import random_genome, simulate_reads, c3_lengths
    want = json.load(open(os.path.join(GOLD, "c3_digest.json")))
    n = want["n_reads"]
    g = random_genome(c3_lengths(), 3000, repeats=(1_000_000, 300, 200, 0.12))
    ix = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0)
    try:
        rb = simulate_reads(g, n, 100, seed=20261015, first=0, sub=0.01, indel=0.001)
        del g
        pk = sa.pack_reads(rb, 100, threads=16)
        del rb
        out, _, _ = ix.vote_packed(default_params(), pk)
        raw = out.view(np.uint8).reshape(n, -1)
        B = want["block_reads"]
        got_blocks = [hashlib.sha256(raw[a:a + B].tobytes()).hexdigest() for a in range(0, n, B)]
        bad = [i for i, (a, b) in enumerate(zip(got_blocks, want["block_sha256"])) if a != b]
        assert not bad, "records differ from the reference in 1M-read blocks %s" % bad[:10]
        assert int((out["selected_votes"][:, 0, 0] > 0).sum()) == want["reads_with_votes"]
    finally:
        ix.close()
