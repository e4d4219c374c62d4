"""GPU EM and assignment (skq_em_*, include/skq.h) against the oracle's
estimate_isoform_abundance_em / assign_reads_to_isoforms (src/isoform_assignment.cpp:9-97).

The posterior sums are added in a different order than the oracle's read order (the reference's
own order is unordered_map iteration order), so pi and counts are compared to a relative 1e-11;
the round count, the set of assigned transcripts and the run-to-run bits are exact.
"""
import random

import numpy as np
import pytest
import torch  # before skq: one HIP runtime per process

import orc
import skq
from skq import synth

pytestmark = pytest.mark.gpu

RTOL = 1e-11


def random_candidates(rng, nreads, ntx, maxc=9, maxs=40):
    offs, tids, scores = [0], [], []
    for _ in range(nreads):
        c = min(ntx, rng.choice([0, 1, 1, 2, 3, 5, maxc]))
        t = rng.sample(range(ntx), c)
        tids += t
        scores += [rng.randint(1, maxs) for _ in t]
        offs.append(len(tids))
    return np.array(offs, np.uint64), np.array(tids, np.uint32), np.array(scores, np.uint32)


def check(em, o, t, s, ntx, max_iterations=20, convergence=0.01):
    pi, it = em.run(max_iterations, convergence)
    pi_ref, it_ref = orc.em(o, t, s, ntx, max_iterations, convergence)
    assert it == it_ref
    np.testing.assert_allclose(pi, pi_ref, rtol=RTOL, atol=0)
    counts, assigned = em.assign()
    c_ref, a_ref = orc.assign(o, t, s, ntx, pi_ref)
    np.testing.assert_array_equal(assigned, a_ref)
    np.testing.assert_allclose(counts, c_ref, rtol=RTOL, atol=1e-300)
    return pi, counts


@pytest.mark.parametrize("nreads,ntx", [(1, 1), (50, 7), (3000, 400), (200_000, 5000), (0, 3)])
def test_em_matches_the_oracle(nreads, ntx):
    rng = random.Random(nreads + ntx)
    o, t, s = random_candidates(rng, nreads, ntx)
    em = skq.EMSet(ntx)
    em.add(o, t, s)
    assert em.reads() == nreads
    check(em, o, t, s, ntx)


def test_em_long_lists_and_many_rounds():
    rng = random.Random(7)
    o, t, s = random_candidates(rng, 20_000, 3000, maxc=200, maxs=300)
    em = skq.EMSet(3000)
    em.add(o, t, s)
    check(em, o, t, s, 3000, max_iterations=100, convergence=1e-9)


def test_appending_in_chunks_and_selecting():
    rng = random.Random(11)
    o, t, s = random_candidates(rng, 5000, 300)
    em = skq.EMSet(300)
    for a, b in [(0, 1), (1, 1000), (1000, 1000), (1000, 4321), (4321, 5000)]:
        em.add(o[a:b + 1], t, s)
    assert em.size() == 5000
    keep = np.array([rng.random() < 0.6 for _ in range(5000)], np.uint8)
    em.select(keep)
    assert em.reads() == int(keep.sum())
    # the oracle on the kept reads only
    ko, kt, ks = [0], [], []
    for r in np.nonzero(keep)[0]:
        kt += list(t[o[r]:o[r + 1]])
        ks += list(s[o[r]:o[r + 1]])
        ko.append(len(kt))
    check(em, np.array(ko, np.uint64), np.array(kt, np.uint32), np.array(ks, np.uint32), 300)


def test_bitwise_reproducible():
    rng = random.Random(5)
    o, t, s = random_candidates(rng, 50_000, 2000)
    a = skq.EMSet(2000)
    a.add(o, t, s)
    b = skq.EMSet(2000)
    b.add(o, t, s)
    pa, ia = a.run()
    pb, ib = b.run()
    assert ia == ib
    assert pa.tobytes() == pb.tobytes()


def test_sharded_rounds_equal_one_device():
    """The multi-GPU EM (skq/dist.py): shards' posterior sums added, then the same M-step; two
    EM sets on one device stand in for two ranks."""
    rng = random.Random(3)
    o, t, s = random_candidates(rng, 30_000, 1500)
    ntx = 1500
    shards = []
    for a, b in [(0, 12_345), (12_345, 30_000)]:
        e = skq.EMSet(ntx)
        e.add(o[a:b + 1], t, s)
        shards.append(e)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    R = sum(e.reads() for e in shards)
    pi = torch.empty(ntx, dtype=torch.float64, device=dev)
    post = torch.empty_like(pi)
    part = torch.empty_like(pi)
    shards[0].init(pi.data_ptr(), st)
    it = 0
    while it < 20:
        post.zero_()
        for e in shards:
            e.estep(pi.data_ptr(), part.data_ptr(), st)
            post += part
        ch = shards[0].mstep(pi.data_ptr(), post.data_ptr(), R, st)
        it += 1
        if ch < 0.01:
            break
    pi_ref, it_ref = orc.em(o, t, s, ntx)
    assert it == it_ref
    np.testing.assert_allclose(pi.cpu().numpy(), pi_ref, rtol=RTOL, atol=0)


@pytest.mark.parametrize("kset", [[31], [21, 25, 31]], ids=["k31", "k21_25_31"])
def test_from_session_results(kset):
    """Candidates appended straight from the session (device to device, the packed candidate
    layout of the fused map at one k slot and with the multi-k passes), two batches, then the
    reference's read filter applied with select."""
    tx = synth.transcriptome(400, seed=9)
    seqs = [tx.seq(i) for i in range(tx.ntx)]
    buf, offs = skq.pack_reads(seqs)
    index = skq.Index(kset, tx.ntx, skq.build_tables(buf, offs, kset))
    bases, _, _ = synth.reads(tx, 6000, 150, seed=10, err=0.002)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(6000)]
    reads[17] = reads[17][:20]                      # short: dropped by the reference
    reads[99] = reads[99][:70] + b"N" + reads[99][71:]  # invalid: dropped
    em = skq.EMSet(tx.ntx)
    s = skq.Session(index, 4000, 150)
    allo, allt, alls, status = [0], [], [], []
    for a, b in [(0, 4000), (4000, 6000)]:
        rb, ro = skq.pack_reads(reads[a:b])
        d_buf = skq.DeviceBuffer.from_numpy(rb)
        d_offs = skq.DeviceBuffer.from_numpy(ro)
        s.map(d_buf.ptr, d_offs.ptr, b - a, 150)
        s.check()
        em.add_session(s)
        out = s.export()
        co = out["cand_offs"]
        for r in range(b - a):
            allt += list(out["cand_tid"][co[r]:co[r + 1]])
            alls += list(out["cand_score"][co[r]:co[r + 1]])
            allo.append(len(allt))
        status += list(out["status"])
    assert em.size() == 6000
    keep = (np.array(status) == skq.READ_OK).astype(np.uint8)
    assert keep[17] == 0 and keep[99] == 0
    em.select(keep)
    ko, kt, ks = [0], [], []
    for r in np.nonzero(keep)[0]:
        kt += allt[allo[r]:allo[r + 1]]
        ks += alls[allo[r]:allo[r + 1]]
        ko.append(len(kt))
    assert len(kt) > 10_000
    check(em, np.array(ko, np.uint64), np.array(kt, np.uint32), np.array(ks, np.uint32), tx.ntx)


def test_out_of_range_transcript_is_an_error():
    em = skq.EMSet(5)
    em.add(np.array([0, 2], np.uint64), np.array([1, 5], np.uint32), np.array([3, 3], np.uint32))
    with pytest.raises(skq.SkqError):
        em.run()


def test_no_reads_after_select():
    em = skq.EMSet(4)
    em.add(np.array([0, 1], np.uint64), np.array([1], np.uint32), np.array([2], np.uint32))
    em.select(np.array([1], np.uint8))
    with pytest.raises(skq.SkqError):
        em.add(np.array([0, 1], np.uint64), np.array([1], np.uint32), np.array([2], np.uint32))


def _dist_em_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    from skq import dist as sdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, t, s = random_candidates(random.Random(21), 20_000, 900)
        start, count = sdist.shard(len(o) - 1, rank, world)
        em = skq.EMSet(900)
        em.add(o[start:start + count + 1], t, s)
        pi, it = sdist.em_gpu(em, 20, 0.01, device=torch.device("cuda", 0))
        counts, assigned = sdist.assign_gpu(em, pi)
        q.put((rank, pi.cpu().numpy(), it, counts.cpu().numpy(), assigned.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_distributed_em_two_ranks():
    """skq/dist.py's em_gpu / assign_gpu with two ranks (processes) on this GPU, gloo standing in
    for RCCL: per-rank E-steps on device, posterior sums all-reduced each round."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_em_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=100) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o, t, s = random_candidates(random.Random(21), 20_000, 900)
    pi_ref, it_ref = orc.em(o, t, s, 900)
    c_ref, a_ref = orc.assign(o, t, s, 900, pi_ref)
    for _, pi, it, counts, assigned in got:
        assert it == it_ref
        np.testing.assert_allclose(pi, pi_ref, rtol=RTOL, atol=0)
        np.testing.assert_allclose(counts, c_ref, rtol=RTOL, atol=1e-300)
        np.testing.assert_array_equal(assigned, a_ref)
    assert got[0][1].tobytes() == got[1][1].tobytes()
