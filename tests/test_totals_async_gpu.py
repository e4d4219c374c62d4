"""skq_session_totals_async (bench.py --gpus N's per-step snapshot): the totals copied on the
session's tail stream after each batch, on a stream of their own, while the next batch's map is
already queued on the launch stream. The same reads map every batch, so the k-th snapshot must be
exactly k times the first, and the last must equal the session's own totals — for batches whose
tail runs on the side stream (4M+ reads, the frames) and for small ones (the launch stream)."""
import numpy as np
import pytest
import torch

import skq
from skq import synth

pytestmark = pytest.mark.gpu

L = 150


@pytest.fixture(scope="module")
def setup():
    tx = synth.transcriptome(3000, seed=61)
    tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=8)
    index = skq.Index([31], tx.ntx, tables, device=0)
    yield tx, index
    index.free()


@pytest.mark.parametrize("n", [100_000, 4_200_000])
def test_async_snapshots_scale_with_the_batches(setup, n):
    tx, index = setup
    bases, _, _ = synth.reads(tx, n, L, seed=62)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(bases).to(dev)
    s = skq.Session(index, n, L)
    main = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev)
    sp = main.cuda_stream
    snaps = [torch.zeros(2, tx.ntx, dtype=torch.int64, device=dev) for _ in range(3)]
    for k in range(3):
        s.map(d.data_ptr(), None, n, L, fixed_len=L, stream=sp, accumulate=True)
        with torch.cuda.stream(comm):
            s.totals_async(snaps[k][0].data_ptr(), snaps[k][1].data_ptr(), stream=comm.cuda_stream)
    torch.cuda.synchronize(dev)
    s.check()
    got = [x.cpu().numpy() for x in snaps]
    final = np.stack(s.totals()).astype(np.int64)
    s.free()
    assert got[0][0].sum() >= n  # (most reads list a candidate)
    for k in range(3):
        np.testing.assert_array_equal(got[k], (k + 1) * got[0])
    np.testing.assert_array_equal(got[2], final)


@pytest.mark.parametrize("n", [100_000, 4_200_000])
def test_results_totals_are_current_after_the_stream(setup, n):
    """skq_session_results folds the batch's packed sums on the stream of the last batch's tail
    (include/skq.h): once that stream is synchronized, the device totals it points at equal
    skq_session_totals' copy."""
    tx, index = setup
    bases, _, _ = synth.reads(tx, n, L, seed=63)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(bases).to(dev)
    s = skq.Session(index, n, L)
    sp = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        s.map(d.data_ptr(), None, n, L, fixed_len=L, stream=sp, accumulate=True)
    r = s.results()
    torch.cuda.synchronize(dev)
    got = []
    for ptr in (r.tx_reads, r.tx_score):
        h = np.zeros(tx.ntx, np.uint64)
        assert skq.lib().skq_memcpy_d2h(h.ctypes.data, ptr, h.nbytes, None) == 0
        got.append(h)
    torch.cuda.synchronize(dev)
    want = s.totals()
    s.free()
    assert got[0].sum() >= 2 * n
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])
