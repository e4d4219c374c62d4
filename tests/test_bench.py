"""bench.py's own checks: the parity comparison it runs on its sample (CPU: a planted difference
in each compared output is reported), and its end_to_end leg (GPU: FASTQ file -> device parse ->
map -> EM, totals equal to the in-HBM map of the same reads)."""
import ctypes as C
import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _outputs():
    """A consistent GPU-export / oracle-output pair for 3 reads, 1 k slot."""
    gpu = {"status": np.array([0, 0, 1], np.uint8),
           "hash_offs": np.array([0, 2, 3, 3], np.uint64), "hashes": np.array([5, 9, 7], np.uint32),
           "cand_offs": np.array([0, 2, 3, 3], np.uint64), "cand_tid": np.array([4, 1, 2], np.uint32),
           "cand_score": np.array([2, 1, 1], np.uint32)}
    cpu = {"n": 3, "status": np.array([0, 0, 1], np.uint8),
           "hash_cnt": np.array([[2], [1], [0]], np.uint32),
           "hashes": np.array([[[5, 9]], [[7, 0]], [[0, 0]]], np.uint32),
           "cand_cnt": np.array([2, 1, 0], np.uint32),
           "cand_tid": np.array([[4, 1], [2, 0], [0, 0]], np.uint32),
           "cand_score": np.array([[2, 1], [1, 0], [0, 0]], np.uint32),
           "tx_reads": np.array([0, 1, 1, 0, 1], np.int64), "tx_score": np.array([0, 1, 1, 0, 2], np.int64)}
    tot = (cpu["tx_reads"].copy(), cpu["tx_score"].copy())
    return gpu, tot, cpu


def test_parity_check_reports_each_planted_difference():
    b = _bench()
    gpu, tot, cpu = _outputs()
    assert b.parity_check(gpu, tot, cpu, 1) == []
    for key, idx, what in [("status", 2, "status"), ("hashes", 1, "retained hashes"),
                           ("cand_tid", 2, "candidate transcripts"), ("cand_score", 0, "candidate scores")]:
        g, t, c = _outputs()
        g[key] = g[key].copy()
        g[key][idx] += 1
        bad = b.parity_check(g, t, c, 1)
        assert bad and bad[0].startswith(what), (key, bad)
    g, t, c = _outputs()
    t[1][4] += 1
    assert b.parity_check(g, t, c, 1) == ["per-transcript totals differ"]
    g, t, c = _outputs()
    g["cand_offs"] = np.array([0, 1, 3, 3], np.uint64)
    assert b.parity_check(g, t, c, 1)[0].startswith("candidate counts")


@pytest.mark.gpu
def test_end_to_end_leg_matches_the_in_hbm_map():
    import torch
    import skq
    from skq import synth
    b = _bench()
    tx = synth.transcriptome(2000, seed=3)
    tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=8)
    index = skq.Index([31], tx.ntx, tables)
    n, L = 300_000, 150
    bases, _, _ = synth.reads(tx, n, L, seed=5, err=0.001)
    d = torch.from_numpy(bases).to("cuda")
    sess = skq.Session(index, n, L)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = b.end_to_end(index, tx.ntx, bases, d.data_ptr(), n, L, sess, sp, batch=100_000)
    assert res["check"] == "totals equal the in-HBM map's, all reads kept", res
    assert res["reads"] == n and res["em_rounds"] >= 1 and res["assigned_transcripts"] > 0
