#!/usr/bin/env python3
"""Per-step times of back-to-back cfg3 maps from a cold start (development tool): an event on the
launch stream after every step, no host sync in between; prints the curve, so the warm-up's
length and cause can be read off (tables, caches, allocation)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import skq  # noqa: E402
from skq import synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
tx = synth.transcriptome(200_000, seed=1)
tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=16)
ix = skq.Index([31], tx.ntx, tables, seqs=(tx.seqs, tx.offs))
n, L = 10_000_000, 150
bases, _, _ = synth.reads(tx, n, L, seed=1000, err=0.001)
d = torch.from_numpy(bases).to("cuda:0")
st = torch.cuda.current_stream()
sp = C.c_void_p(st.cuda_stream)
s = skq.Session(ix, n, L)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
ev[0].record(st)
for i in range(steps):
    s.map(d.data_ptr(), None, n, L, fixed_len=L, stream=sp)
    ev[i + 1].record(st)
torch.cuda.synchronize()
t = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)])
print("per-step ms:", " ".join("%.3f" % x for x in t))
for a, b in ((0, 5), (5, 10), (10, 20), (20, 30), (30, 45), (45, steps)):
    if a < steps:
        print("steps %2d-%2d: mean %.4f ms" % (a, min(b, steps), t[a:b].mean()))
