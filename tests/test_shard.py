"""Multi-GPU path on the CPU: reads sharded over world_size 2 (gloo), each rank
votes its contiguous shard, rank 0 gathers the records in read order, and the
result is byte-identical to the reference's golden records for the whole batch.
The vote function here is the oracle (test infrastructure); on GPUs each rank
calls its own HIP index replica the same way (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.common import Case, ensure_built, pack_records

ensure_built()


def test_shard_range_covers_exactly():
    from subread_amd.shard import shard_range
    for n in (0, 1, 7, 8, 1000, 1001):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, r, w) for r in range(w)]
            assert sum(c for _, c in got) == n
            assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(w - 1))
            assert max(c for _, c in got) - min(c for _, c in got) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, prefix, case, out_path):
    import torch.distributed as dist
    from oracle.pyoracle import OracleIndex
    from subread_amd.shard import vote_sharded
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        c = Case(case)
        oi = OracleIndex(prefix)

        def vote(a, b):
            out, jout, bm, _ = oi.vote(c.params, a, b, threads=2)
            return out, jout, bm
        res = vote_sharded(vote, c.r1, c.r2)
        if rank == 0:
            np.save(out_path, pack_records(*res))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["pe_full_errmut", "sj_se_full_junc"])
def test_two_rank_gloo_shards_match_golden(case, index_cache, tmp_path):
    c = Case(case)
    prefix = index_cache.get(c.index_key)
    out_path = str(tmp_path / "gathered.npy")
    mp.start_processes(_rank_main, args=(2, _free_port(), prefix, case, out_path), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out_path)
    assert got.shape == c.expected.shape
    assert (got == c.expected).all()
