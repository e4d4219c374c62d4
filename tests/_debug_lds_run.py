"""Run by tests/test_debug_lds_gpu.py in a child process with SKQ_LIB pointing at the debug build
(make debuglds: the map's LDS slot counter clamped at 0 instead of wrapping below LDS address 0):
one k = 31 batch (k_map1) and one k = {21, 25, 31} batch (the passes; the k = 21 pass's 16 rows
overflow on ~0.2 % of the reads, so lanes run past row 0), each per read against the oracle."""
import os
import sys

import numpy as np
import torch  # noqa: F401  (before skq: one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import digest  # noqa: E402
import orc  # noqa: E402
import skq  # noqa: E402
from skq import synth  # noqa: E402

assert skq.LIB_PATH == os.environ["SKQ_LIB"], skq.LIB_PATH
tx = synth.transcriptome(20_000, seed=5)
n, L = 300_000, 150
bases, _, _ = synth.reads(tx, n, L, seed=6, err=0.001)
d = skq.DeviceBuffer.from_numpy(bases)
for ks in ([31], [21, 25, 31]):
    tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
    index = skq.Index(ks, tx.ntx, tables, seqs=(tx.seqs, tx.offs))
    pairs = []
    for k in ks:
        keys, offs, tids = tables[k]
        pairs.append((np.repeat(keys, np.diff(offs.astype(np.int64))), tids))
    cpu = orc.map_digest(orc.Index(ks, pairs=pairs, ntx=tx.ntx), bases, L, nthreads=16)
    s = skq.Session(index, n, L)
    s.map(d.ptr, None, n, L, fixed_len=L)
    s.check()
    dg = digest.export_digest(s.export(), len(ks))
    tot = s.totals()
    slow = s.slow_reads()
    s.free()
    index.free()
    bad = np.nonzero(dg != cpu["digest"])[0]
    assert len(bad) == 0, "ks=%s: %d reads differ (first %s)" % (ks, len(bad), bad[:8].tolist())
    assert np.array_equal(tot[0], cpu["tx_reads"]) and np.array_equal(tot[1], cpu["tx_score"]), ks
    print("ks=%s: %d reads per read bit-exact, slow reads %s" % (ks, n, slow), flush=True)
d.free()
print("debug-lds ok")
