"""RCCL itself on the GPU (the multi-GPU paths' library calls, on a one-GPU box):
  * the skq CLI's sharded EM over a one-rank RCCL communicator (SKQ_REDUCE=rccl: ncclCommInitAll
    over one device, grouped in-place ncclAllReduce of the double posterior sums and the
    ncclUint8 / ncclMax assigned flags) gives the single-device CSV;
  * skq/dist.py under a world-1 "nccl" process group: the per-transcript totals all-reduce and the
    sharded EM / assignment (em_gpu, assign_gpu) run through RCCL and equal the oracle's;
  * a FASTQ of two records split four ways (parts with no records) quantifies like one part."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import orc
from skq import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "skq")


def _run(*args, env=None):
    import subprocess
    return subprocess.run([CLI, *map(str, args)], check=True, capture_output=True, text=True, timeout=300,
                          env=env).stdout


def _rows(path):
    lines = open(path).read().splitlines()
    assert lines[0] == "Name,NumReads,EM_Abundance"
    return {l.split(",")[0]: (float(l.split(",")[1]), float(l.split(",")[2])) for l in lines[1:]}


def _fixture(tmp_path, ntx=150, nreads=3000, seed=81):
    tx = synth.transcriptome(ntx, seed=seed)
    fa, fq = tmp_path / "t.fa", tmp_path / "r.fq"
    tx.write_fasta(fa)
    bases, _, _ = synth.reads(tx, nreads, 150, seed=seed + 1)
    fq.write_bytes(synth.fastq_bytes(bases, 150).tobytes())
    idx = tmp_path / "t.idx"
    _run("-k", "31", "-o", "index", fa, idx)
    return tx, fa, fq, idx


def test_cli_rccl_one_rank_communicator(tmp_path):
    _, _, fq, idx = _fixture(tmp_path)
    one, rccl = tmp_path / "one.csv", tmp_path / "rccl.csv"
    _run("-o", "quant", idx, fq, one)
    _run("-o", "quant", idx, fq, rccl, env=dict(os.environ, SKQ_DEVICES="0", SKQ_REDUCE="rccl"))
    a, b = _rows(one), _rows(rccl)
    assert set(a) == set(b) and len(a) > 100
    for t in a:  # one rank: the same sums in the same order as the single-device EM
        assert b[t] == pytest.approx(a[t], rel=2e-6), t


def test_cli_parts_without_records(tmp_path):
    """parts that hold no records (a tiny FASTQ split four ways) have no kept array."""
    tx, _, _, idx = _fixture(tmp_path, nreads=10)
    fq2 = tmp_path / "two.fq"
    bases, _, _ = synth.reads(tx, 2, 150, seed=99)
    fq2.write_bytes(synth.fastq_bytes(bases, 150).tobytes())
    one, four = tmp_path / "one.csv", tmp_path / "four.csv"
    _run("-o", "quant", idx, fq2, one)
    _run("-o", "quant", idx, fq2, four, env=dict(os.environ, SKQ_DEVICES="0,0,0,0"))
    a, b = _rows(one), _rows(four)
    assert set(a) == set(b) and len(a) >= 1
    for t in a:
        assert b[t] == pytest.approx(a[t], rel=2e-6), t


def _worker(port, q):
    import torch.distributed as dist
    import skq
    from skq import dist as sdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        tx = synth.transcriptome(2000, seed=91)
        tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=4)
        index = skq.Index([31], tx.ntx, tables, device=0)
        n, L = 40_000, 150
        bases, _, _ = synth.reads(tx, n, L, seed=92)
        d = torch.from_numpy(bases).to(dev)
        s = skq.Session(index, n, L)
        s.map(d.data_ptr(), None, n, L, fixed_len=L)
        s.check()
        totals = torch.zeros(2, tx.ntx, dtype=torch.int64, device=dev)
        s.totals_to_device(totals[0].data_ptr(), totals[1].data_ptr())
        torch.cuda.synchronize()
        sdist.allreduce_totals(totals)  # through RCCL (world 1)
        out = s.export()
        em = skq.EMSet(tx.ntx, device=0)
        em.add_session(s)
        pi, it = sdist.em_gpu(em, 20, 0.01, device=dev)
        counts, assigned = sdist.assign_gpu(em, pi)
        torch.cuda.synchronize()
        q.put(dict(backend=dist.get_backend(), totals=totals.cpu().numpy(), pi=pi.cpu().numpy(), it=it,
                   counts=counts.cpu().numpy(), assigned=assigned.cpu().numpy(), cand_offs=out["cand_offs"],
                   cand_tid=out["cand_tid"], cand_score=out["cand_score"], bases=bases, ntx=tx.ntx,
                   tables=tables))
        em.free()
    finally:
        dist.destroy_process_group()


def test_world1_nccl_totals_and_em():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, q))
    p.start()
    r = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert r["backend"] == "nccl"
    keys, offs, tids = r["tables"][31]
    oi = orc.Index([31], pairs=[(np.repeat(keys, np.diff(offs.astype(np.int64))), tids)], ntx=r["ntx"])
    cpu = orc.fastq_map(oi, synth.fastq_bytes(r["bases"], 150), nthreads=8, outputs=False, totals=True)
    np.testing.assert_array_equal(r["totals"][0], cpu["tx_reads"])
    np.testing.assert_array_equal(r["totals"][1], cpu["tx_score"])
    pi_ref, it_ref = orc.em(r["cand_offs"], r["cand_tid"], r["cand_score"], r["ntx"])
    c_ref, a_ref = orc.assign(r["cand_offs"], r["cand_tid"], r["cand_score"], r["ntx"], pi_ref)
    assert r["it"] == it_ref
    np.testing.assert_allclose(r["pi"], pi_ref, rtol=1e-11, atol=0)
    np.testing.assert_allclose(r["counts"], c_ref, rtol=1e-11, atol=1e-300)
    np.testing.assert_array_equal(r["assigned"], a_ref.astype(bool))
