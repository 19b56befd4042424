"""CPU: the oracle restatement (oracle/svoracle.c) reproduces the reference's own
vote records byte for byte on every golden fixture (tests/golden/make_golden.py),
on indexes built by OUR format-exact builder (md5-checked against the reference)."""
import pytest

from tests.common import Case, golden_names, ensure_built, pack_records, describe_mismatch

ensure_built()


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference(name, index_cache):
    from oracle.pyoracle import OracleIndex
    c = Case(name)
    ix = OracleIndex(index_cache.get(c.index_key))
    out, jout, bm, st = ix.vote(c.params, c.r1, c.r2, threads=4)
    got = pack_records(out, jout, bm)
    assert got.shape == c.expected.shape
    ok = (got == c.expected).all()
    assert ok, describe_mismatch(got, c.expected, c.ends, c.params.multi_best)
