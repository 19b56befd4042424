"""Multi-GPU sharding of the vote path.

The unit of work is the read (SE) or the pair (PE): voting depends only on the
read and the read-only index.  Each rank (one process per GPU) holds a full
index replica and votes one contiguous range of the batch; there is no
collective on the data path.  The host puts the records back in read order
(the reference's equivalent is the per-chunk bigtable, core-bigtable.c:84-131,
which later feeds the SAM writer in read order).

`gather_records` uses torch.distributed only to move finished host records to
one rank; bench.py does not gather at all (it times the vote step).
"""
import numpy as np


def shard_range(n_total, rank, world):
    """Contiguous, balanced [first, first+count) of n_total units for `rank`."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world %r/%r" % (rank, world))
    base, extra = divmod(int(n_total), int(world))
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def gather_records(local, dst=0, group=None):
    """Concatenate every rank's record array in rank order on `dst` (None elsewhere)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(local, parts, dst=dst, group=group)
    if parts is None:
        return None
    return tuple(np.concatenate([p[k] for p in parts], 0) if parts[0][k] is not None else None
                 for k in range(len(parts[0])))


def vote_sharded(vote, r1, r2=None, dst=0, group=None):
    """Vote this rank's shard of (r1, r2) with `vote(r1_part, r2_part)` -> tuple of record
    arrays (first axis = read), then gather them on `dst` in read order."""
    import torch.distributed as dist
    first, count = shard_range(len(r1), dist.get_rank(group), dist.get_world_size(group))
    a = r1.slice(first, first + count)
    b = r2.slice(first, first + count) if r2 is not None else None
    return gather_records(vote(a, b), dst=dst, group=group)
