"""The multi-GPU layer (skq/dist.py) with world_size 2 on gloo: sharding covers every read once,
and the all-reduced per-transcript totals of the shards equal those of the whole batch. The
per-shard work here is the oracle (CPU); on GPUs it is skq_map on each rank's device."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import orc
from skq import dist as sdist
from skq import synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partitions_reads():
    for n in (0, 1, 7, 100, 10_000_001):
        for w in (1, 2, 3, 8):
            spans = [sdist.shard(n, r, w) for r in range(w)]
            assert sum(c for _, c in spans) == n
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _totals(ref, lo, hi, ntx):
    out = np.zeros((2, ntx), np.int64)
    for r in range(lo, hi):
        c = ref["cand_cnt"][r]
        for j in range(c):
            out[0, ref["cand_tid"][r, j]] += 1
            out[1, ref["cand_tid"][r, j]] += ref["cand_score"][r, j]
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = synth.transcriptome(80, seed=31)
        seqs = [tx.seq(t) for t in range(tx.ntx)]
        bases, _, _ = synth.reads(tx, 301, 150, seed=32)
        reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(301)]
        start, count = sdist.shard(len(reads), *sdist.world()[:2])
        ref = orc.Index([31], seqs=seqs).map_batch(reads[start:start + count])
        mine = torch.from_numpy(_totals(ref, 0, count, tx.ntx))
        sdist.allreduce_totals(mine)
        slowest = sdist.max_over_ranks(0.5 + rank)
        q.put((rank, mine.numpy(), slowest))
    finally:
        dist.destroy_process_group()


def test_allreduced_shard_totals_equal_whole_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tx = synth.transcriptome(80, seed=31)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    bases, _, _ = synth.reads(tx, 301, 150, seed=32)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(301)]
    whole = _totals(orc.Index([31], seqs=seqs).map_batch(reads), 0, 301, tx.ntx)
    assert whole[0].sum() > 200
    for rank, tot, slowest in got:
        np.testing.assert_array_equal(tot, whole)
        assert slowest == 1.5


def _em_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, t, s = _em_candidates()
        start, count = sdist.shard(len(o) - 1, rank, world)
        so = o[start:start + count + 1] - o[start]
        st = t[o[start]:o[start + count]]
        ss = s[o[start]:o[start + count]]
        pi, it = sdist.em_host(so, st, ss, 700)
        q.put((rank, pi, it))
    finally:
        dist.destroy_process_group()


def _em_candidates():
    rng = np.random.default_rng(77)
    cnt = rng.choice([0, 1, 1, 2, 3, 5, 9], size=4001)
    offs = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
    tids = np.concatenate([rng.choice(700, size=c, replace=False) for c in cnt]).astype(np.uint32)
    scores = rng.integers(1, 40, size=len(tids)).astype(np.uint32)
    return offs, tids, scores


def test_sharded_em_equals_whole_batch():
    """The EM over read shards (skq/dist.py: per-rank E-step, all-reduced posterior sums, the
    M-step on every rank) against the oracle EM over all reads, world size 2 on gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_em_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=240) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o, t, s = _em_candidates()
    pi_ref, it_ref = orc.em(o, t, s, 700)
    for _, pi, it in got:
        assert it == it_ref
        # shards add their posterior sums separately: only the order of additions differs
        np.testing.assert_allclose(pi, pi_ref, rtol=1e-12, atol=0)
    assert got[0][1].tobytes() == got[1][1].tobytes()  # every rank holds the same pi
