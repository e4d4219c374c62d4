"""The multi-GPU map on the GPU: two ranks (processes) on this one GPU, each running skq_map over
its read shard through the C ABI, the per-transcript totals copied to device tensors and
all-reduced (skq/dist.py; gloo stands in for RCCL on one GPU). The reduced totals equal the
oracle's over the whole batch, on every rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import orc
from skq import synth

pytestmark = pytest.mark.gpu

NTX, NREADS, L = 3000, 60_001, 150


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import skq
    from skq import dist as sdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = synth.transcriptome(NTX, seed=41)
        tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=4)
        index = skq.Index([31], tx.ntx, tables, device=0)
        bases, _, _ = synth.reads(tx, NREADS, L, seed=42)
        start, count = sdist.shard(NREADS, rank, world)
        d = torch.from_numpy(bases[start * L:(start + count) * L]).to(dev)
        s = skq.Session(index, count, L)
        totals = torch.zeros(2, tx.ntx, dtype=torch.int64, device=dev)
        for _ in range(2):  # two steps: the totals accumulate in the session
            s.map(d.data_ptr(), None, count, L, fixed_len=L)
        s.check()
        s.totals_to_device(totals[0].data_ptr(), totals[1].data_ptr())
        torch.cuda.synchronize()
        sdist.allreduce_totals(totals)
        q.put((rank, totals.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_map_totals_equal_the_oracle():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=100) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tx = synth.transcriptome(NTX, seed=41)
    import skq
    tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=4)
    keys, offs, tids = tables[31]
    oi = orc.Index([31], pairs=[(np.repeat(keys, np.diff(offs.astype(np.int64))), tids)], ntx=tx.ntx)
    bases, _, _ = synth.reads(tx, NREADS, L, seed=42)
    cpu = orc.fastq_map(oi, synth.fastq_bytes(bases, L), nthreads=8, outputs=False, totals=True)
    for _, t in got:
        np.testing.assert_array_equal(t[0], 2 * cpu["tx_reads"].astype(np.int64))
        np.testing.assert_array_equal(t[1], 2 * cpu["tx_score"].astype(np.int64))
    assert int(got[0][1][0].sum()) > 2 * NREADS
