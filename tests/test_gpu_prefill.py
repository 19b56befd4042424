"""svg_probe_keys (cellCounts' prefill_votes on the GPU, cell-counts.c:432-491) through the C ABI:
bit-exact against the reference's own outputs (tests/golden/prefill/prefill.npz) on full, gapped
and multi-block indexes, and against the oracle restatement on 2M keys (genome 16-mers from
repeat-rich synth4242, random keys, edge keys)."""
import os

import numpy as np
import pytest

from tests.common import GOLD, ensure_built

ensure_built()
pytestmark = pytest.mark.gpu
FIX = os.path.join(GOLD, "prefill", "prefill.npz")
INDEXES = ["chr901_full", "chr901_gapped", "synth4242_full", "synth4242_gapped", "synth4242_fullM1"]


@pytest.mark.parametrize("key", INDEXES)
def test_gpu_probe_keys_matches_reference(key, index_cache):
    import subread_amd as sa
    z = np.load(FIX, allow_pickle=False)
    keys, block = z[key + "_keys"], int(z[key + "_block"][0])
    ix = sa.VoteIndex(index_cache.get(key), device=0)
    f, c = ix.probe_keys(keys, block)
    ix.close()
    assert (c == z[key + "_count"]).all()
    assert (f == z[key + "_first"]).all()


def test_gpu_probe_keys_matches_oracle_at_scale(index_cache):
    import subread_amd as sa
    from oracle.pyoracle import OracleIndex
    from subread_amd.sim import Genome
    key = "synth4242_full"
    pre = index_cache.get(key)
    g = Genome.read_fasta(index_cache.genome_fasta("synth4242"))
    rng = np.random.default_rng(7)
    code = np.full(256, 3, np.uint32)
    code[ord("A")], code[ord("G")], code[ord("C")] = 0, 1, 2
    pos = rng.integers(0, len(g.flat) - 16, 1_500_000)
    k = np.zeros(len(pos), np.uint64)
    for i in range(16):
        k = (k << np.uint64(2)) | code[g.flat[pos + i]].astype(np.uint64)
    keys = np.concatenate([k.astype(np.uint32), rng.integers(0, 2 ** 32, 500_000, dtype=np.uint64).astype(np.uint32),
                           np.array([0, 1, 0xffffffff, 0x7fffffff, 0x80000000], np.uint32)])
    ix = sa.VoteIndex(pre, device=0)
    f, c = ix.probe_keys(keys)
    e0, e1 = ix.probe_keys(np.zeros(0, np.uint32))
    ix.close()
    rf, rc = OracleIndex(pre).prefill(keys)
    assert len(e0) == 0 and len(e1) == 0
    assert (c == rc).all() and (f == rf).all()
    assert (c > 0).sum() > 1_000_000
