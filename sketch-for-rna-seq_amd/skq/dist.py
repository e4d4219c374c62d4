"""Multi-GPU layer: one process per GPU (torch.distributed.run), reads sharded, index replicated.

The hot path has no exchange between ranks; the only collective is one all-reduce of the
per-transcript totals (read count, score sum: int64[2, ntx]) per batch over RCCL/xGMI
("nccl" backend), or gloo on CPU for tests. SURVEY.md §8(e).
"""
import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n, rank, world_size):
    """Contiguous shard [start, start + count) of n reads for `rank`; shard sizes differ by at
    most one read and their union is 0..n in rank order."""
    base, extra = divmod(n, world_size)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def allreduce_totals(totals):
    """Sum a [2, ntx] int64 tensor of per-transcript totals over all ranks, in place. A no-op
    without an initialised process group (single GPU)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(totals, op=dist.ReduceOp.SUM)
    return totals


def max_over_ranks(value, device=None):
    """The maximum of a float over ranks (the slowest rank's elapsed time)."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
