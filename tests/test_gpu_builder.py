"""GPU index builder: the index built in HBM is item-for-item the reference's
(files written from it are md5-identical to subread-buildindex's)."""
import os

import numpy as np
import pytest

from tests.common import ensure_built, index_md5, index_recipe, is_multi_block_key, md5

ensure_built()
pytestmark = pytest.mark.gpu


# the in-HBM builder makes one-block indexes (multi-block ones come from the CPU builder)
@pytest.mark.parametrize("key", sorted(k for k in index_md5()["md5"] if not is_multi_block_key(k)))
def test_gpu_built_index_md5(key, index_cache, tmp_path):
    import subread_amd as sa
    gname, gap, memory_mb, force = index_recipe(key)
    fa = index_cache.genome_fasta(gname)
    pre = str(tmp_path / key)
    ix = sa.VoteIndex.build(fa, gap=gap, memory_mb=memory_mb, force_one_block=force, device=0, save_prefix=pre)
    want = index_md5()["md5"][key]
    for suf, m in want.items():
        assert md5(pre + suf) == m, (key, suf)
    # the in-HBM copy equals what svg_index_open would load
    ref = sa.VoteIndex(index_cache.get(key), device=0)
    a, b = ix.export(), ref.export()
    for f in ("bstart", "keys", "vals", "chr_end"):
        assert (a[f] == b[f]).all(), f
    assert (a["values"][:a["values_bytes"]] == b["values"][:b["values_bytes"]]).all()
    ix.close()
    ref.close()


def test_gpu_built_index_votes_identically(index_cache):
    import subread_amd as sa
    from tests.common import Case, pack_records
    c = Case("pe_full_synth")
    ix = sa.VoteIndex.build(index_cache.genome_fasta("synth4242"), gap=1, memory_mb=100, force_one_block=True,
                            device=0)
    out, _, _ = ix.vote(c.params, c.r1, c.r2)
    assert (pack_records(out, None, None) == c.expected).all()
    ix.close()


def test_index_open_from_files_equals_built_index(tmp_path):
    """svg_index_open's streamed load (parallel bucket-chain walk, ~4M-item staging runs on 16
    streams) of a 60 Mbp index (~60M items: many staging runs, repeat-family buckets) gives the
    same arrays in HBM as the index built there, array for array."""
    import subread_amd as sa
    from subread_amd.sim import random_genome
    g = random_genome([25_000_000, 20_000_000, 15_000_000], 606, repeats=(20_000, 300, 40, 0.12))
    pre = str(tmp_path / "g60")
    built = sa.VoteIndex.build_genome(g, gap=1, memory_mb=8000, force_one_block=True, device=0, save_prefix=pre)
    opened = sa.VoteIndex(pre, device=0)
    a, b = built.export(), opened.export()
    assert a["items"] > 50_000_000
    for f in ("bstart", "keys", "vals", "chr_end"):
        assert (a[f] == b[f]).all(), f
    assert (a["values"][:a["values_bytes"]] == b["values"][:b["values_bytes"]]).all()
    built.close()
    opened.close()


def test_index_open_reports_a_missing_array_file(index_cache, tmp_path):
    """svg_index_open loads the .array and contig table on a thread of its own; a failure there comes
    back with its own message (svg_last_error is per thread), not a stale or empty one."""
    import shutil
    import subread_amd as sa
    src = index_cache.get("chr901_gapped")
    pre = str(tmp_path / "noarray")
    for suf in (".00.b.tab", ".reads", ".files"):
        if os.path.exists(src + suf):
            shutil.copy(src + suf, pre + suf)
    with pytest.raises(sa.SvgError) as e:
        sa.VoteIndex(pre, device=0)
    assert ".array" in str(e.value), str(e.value)


@pytest.mark.parametrize("key", ["chr901_full", "synth4242_gappedM1"])
def test_index_open_devices_replicas_equal_single_open(key, index_cache):
    """svg_index_open_devices (the drop-in's several handles): three replicas on device 0 from one
    read of the files, each array equal to a single svg_index_open's, each voting the golden
    records (multi-block index included)."""
    import subread_amd as sa
    from tests.common import Case, pack_records
    pre = index_cache.get(key)
    one = sa.VoteIndex(pre, device=0)
    reps = sa.VoteIndex.open_devices(pre, [0, 0, 0])
    a = one.export()
    for r in reps:
        assert r.n_blocks == one.n_blocks
        b = r.export()
        for f in ("bstart", "keys", "vals", "chr_end"):
            assert (a[f] == b[f]).all(), f
        assert (a["values"][:a["values_bytes"]] == b["values"][:b["values_bytes"]]).all()
    cases = [n for n in ("pe_gapped_errmut", "se_full_errmut", "pe_mb_synth_gappedM1") if Case(n).index_key == key]
    for name in cases:
        c = Case(name)
        for r in reps:
            out, _, _ = r.vote(c.params, c.r1, c.r2)
            assert (pack_records(out, None, None) == c.expected).all(), name
    for r in reps + [one]:
        r.close()
