#!/usr/bin/env python3
"""Development check: multi-k totals of one in-HBM batch against the same reads mapped as
several batches (fixed length / with offsets) and through the FASTQ ingest."""
import os
import sys
import tempfile
import ctypes as C

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import skq  # noqa: E402
from skq import synth  # noqa: E402

ntx = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 400_000
ks = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "21,25,31").split(",")]
L = 150
tx = synth.transcriptome(ntx, seed=1)
tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
index = skq.Index(ks, tx.ntx, tables)
bases, _, _ = synth.reads(tx, N, L, seed=1000, err=0.001)
d = skq.DeviceBuffer.from_numpy(bases)


def tot(s):
    t = s.totals()
    return np.stack(t).astype(np.int64)


s = skq.Session(index, N, L)
s.map(d.ptr, None, N, L, fixed_len=L)
s.check()
A = tot(s)
print("A one batch: candidates", int(A[0].sum()), "slow", s.slow_reads())
s.free()
for B in [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "100000,65536,4096").split(",")]:
    s = skq.Session(index, B, 256)
    for a in range(0, N, B):
        m = min(B, N - a)
        s.map(C.c_void_p(d.ptr.value + a * L), None, m, L, fixed_len=L)
    s.check()
    T = tot(s)
    print("fixed batches of", B, "equal" if np.array_equal(T, A) else "DIFFER %d tx" % int((T != A).any(0).sum()))
    s.free()
offs = (np.arange(N + 1, dtype=np.uint64) * L)
do = skq.DeviceBuffer.from_numpy(offs)
for B in (100_000,):
    s = skq.Session(index, B, 256)
    for a in range(0, N, B):
        m = min(B, N - a)
        o = skq.DeviceBuffer.from_numpy((offs[a:a + m + 1] - offs[a]).astype(np.uint64))
        s.map(C.c_void_p(d.ptr.value + a * L), o.ptr, m, L)
        o.free()
    s.check()
    T = tot(s)
    print("offset batches of", B, "equal" if np.array_equal(T, A) else "DIFFER %d tx" % int((T != A).any(0).sum()))
    s.free()
fd, path = tempfile.mkstemp(suffix=".fq", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
os.close(fd)
with open(path, "wb") as f:
    f.write(synth.fastq_bytes(bases, L).tobytes())
s = skq.Session(index, 2_000_000, 256)
g = skq.Ingest(s, path)
while True:
    _, got = g.map()
    if got == 0:
        break
s.check()
g.finish()
g.close()
T = tot(s)
print("ingest", "equal" if np.array_equal(T, A) else "DIFFER %d tx" % int((T != A).any(0).sum()))
os.unlink(path)
