"""cellCounts' hit-list lookup (prefill_votes, cell-counts.c:432-491): the oracle restatement
(oracle/svoracle.c svo_prefill) against the reference's own prefill_votes outputs
(tests/golden/prefill/prefill.npz, made by oracle/_ref/ref-prefill from the reference source),
on full, gapped and multi-block indexes; the GPU entry (svg_probe_keys) is tested against the
same vectors in test_gpu_prefill.py."""
import os

import numpy as np
import pytest

from tests.common import GOLD, ensure_built

ensure_built()
FIX = os.path.join(GOLD, "prefill", "prefill.npz")
INDEXES = ["chr901_full", "chr901_gapped", "synth4242_full", "synth4242_gapped", "synth4242_fullM1"]


@pytest.mark.parametrize("key", INDEXES)
def test_oracle_prefill_matches_reference(key, index_cache):
    from oracle.pyoracle import OracleIndex
    z = np.load(FIX, allow_pickle=False)
    keys, block = z[key + "_keys"], int(z[key + "_block"][0])
    f, c = OracleIndex(index_cache.get(key)).prefill(keys, block)
    assert (c == z[key + "_count"]).all()
    assert (f == z[key + "_first"]).all()
    assert (c > 0).sum() > 500            # the vectors exercise present keys and long runs
