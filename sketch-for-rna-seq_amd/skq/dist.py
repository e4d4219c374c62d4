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
    without an initialised process group (single GPU); with one, the collective runs at any world
    size (a world-1 RCCL group exercises the library path, tests/test_rccl_gpu.py)."""
    return _allreduce(totals)


def max_over_ranks(value, device=None):
    """The maximum of a float over ranks (the slowest rank's elapsed time)."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _allreduce(t, op=None):
    """Sum (or op) over ranks in place. RCCL takes device tensors directly; on gloo (CPU tests and
    one-GPU rehearsals) a device tensor goes through host memory."""
    if dist.is_available() and dist.is_initialized():
        op = dist.ReduceOp.SUM if op is None else op
        if t.is_cuda and dist.get_backend() == "gloo":
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)
    return t


def _em_loop(estep, post, mstep, max_iterations, convergence):
    """estimate_isoform_abundance_em's rounds (src/isoform_assignment.cpp:23-65) over read shards:
    every rank forms its shard's posterior sums, they are summed over ranks (the one exchange of
    the EM, double[ntx] per round), and the M-step then runs identically on every rank, so every
    rank sees the same change and leaves the loop in the same round."""
    it = 0
    while it < max_iterations:
        estep()
        _allreduce(post)
        change = mstep()
        it += 1
        if change < convergence:
            break
    return it


def em_gpu(emset, max_iterations=20, convergence=0.01, device=None):
    """GPU EM over read shards: emset (skq.EMSet) holds this rank's reads on `device`; post is
    all-reduced over RCCL/xGMI each round. Returns (pi tensor on device, iterations)."""
    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream(device).cuda_stream
    R = _allreduce(torch.tensor([emset.reads()], dtype=torch.int64, device=device))
    total = int(R.item())
    pi = torch.empty(emset.ntx, dtype=torch.float64, device=device)
    post = torch.empty_like(pi)
    emset.init(pi.data_ptr(), stream)
    it = _em_loop(lambda: emset.estep(pi.data_ptr(), post.data_ptr(), stream), post,
                  lambda: emset.mstep(pi.data_ptr(), post.data_ptr(), total, stream), max_iterations, convergence)
    return pi, it


def assign_gpu(emset, pi):
    """assign_reads_to_isoforms over read shards: (counts, assigned) summed / or-ed over ranks."""
    stream = torch.cuda.current_stream(pi.device).cuda_stream
    counts = torch.empty_like(pi)
    assigned = torch.empty(emset.ntx, dtype=torch.uint8, device=pi.device)
    emset.assign_device(pi.data_ptr(), counts.data_ptr(), assigned.data_ptr(), stream)
    _allreduce(counts)
    a32 = assigned.to(torch.int32)
    _allreduce(a32, dist.ReduceOp.MAX)
    return counts, a32.bool()


def em_host(cand_offs, cand_tid, cand_score, ntx, max_iterations=20, convergence=0.01):
    """The same loop with host E-/M-steps (CPU ranks, gloo): (pi numpy, iterations)."""
    import numpy as np
    import skq
    R = _allreduce(torch.tensor([len(cand_offs) - 1], dtype=torch.int64))
    total = int(R.item())
    pi = np.full(ntx, 1.0 / ntx, np.float64)
    post = torch.zeros(ntx, dtype=torch.float64)

    def estep():
        post.copy_(torch.from_numpy(skq.em_estep_host(cand_offs, cand_tid, cand_score, ntx, pi)))

    it = _em_loop(estep, post, lambda: skq.em_mstep_host(pi, post.numpy(), total), max_iterations, convergence)
    return pi, it
