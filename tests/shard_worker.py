"""Worker of tests/test_gpu_shard.py, launched by torch.distributed.run (one process per
rank, gloo for the host-side gather).  Every rank opens its own replica of the index on
GPU `--device` and votes its contiguous shard through the HIP library (the packed host
entry point); rank 0 saves the gathered records."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("case")
    ap.add_argument("out")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    import numpy as np
    import torch.distributed as dist
    import subread_amd as sa
    from subread_amd.shard import vote_sharded
    from tests.common import Case, pack_records
    dist.init_process_group("gloo")
    try:
        c = Case(a.case)
        ix = sa.VoteIndex(a.prefix, device=a.device)

        def vote(r1, r2):
            return ix.vote_packed(c.params, sa.pack_reads(r1), sa.pack_reads(r2) if r2 is not None else None)
        res = vote_sharded(vote, c.r1, c.r2)
        ix.close()
        if dist.get_rank() == 0:
            np.save(a.out, pack_records(*res))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
