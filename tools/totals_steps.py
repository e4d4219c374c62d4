#!/usr/bin/env python3
"""Step time of back-to-back cfg3 batches with the per-transcript totals (development tool): the
bench's own loop shape (skq_map with accumulate over one device-resident batch, K steps between
two syncs), for the totals variant the environment selects (SKQ_TOTALS_FORK, SKQ_MAP_BINS,
SKQ_BIN_BITS ...). Prints ms per step and the map kernel's own time; run it under
rocprofv3 --kernel-trace --stats for the per-kernel durations."""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import skq  # noqa: E402
from skq import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ntx", type=int, default=200_000)
ap.add_argument("--reads", type=int, default=10_000_000)
ap.add_argument("--len", type=int, default=150)
ap.add_argument("--ks", default="31")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--variants", default="", help="K=V[+K=V],... env sets run in turn (interleaved rounds)")
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
tx = synth.transcriptome(a.ntx, seed=1)
ks = [int(x) for x in a.ks.split(",")]
tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
ix = skq.Index(ks, tx.ntx, tables, seqs=(tx.seqs, tx.offs))
bases, _, _ = synth.reads(tx, a.reads, a.len, seed=1000, err=0.001)
d = torch.from_numpy(bases).to("cuda:0")
sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
variants = [dict(kv.split("=", 1) for kv in v.split("+") if kv) for v in a.variants.split(",")] if a.variants else [{}]
keys = sorted({k for v in variants for k in v})
sessions = []
for v in variants:  # (a session per variant: some switches, e.g. SKQ_BIN_BITS, are read at its creation)
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(v)
    sessions.append(skq.Session(ix, a.reads, a.len))
res = {i: [] for i in range(len(variants))}
ref = None
for rnd in range(a.rounds + 1):
    for i, v in enumerate(variants):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(v)
        s = sessions[i]
        s.reset_totals(sp)
        for _ in range(2):
            s.map(d.data_ptr(), None, a.reads, a.len, fixed_len=a.len, stream=sp, accumulate=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            s.map(d.data_ptr(), None, a.reads, a.len, fixed_len=a.len, stream=sp, accumulate=True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / a.steps
        s.check(sp)
        tot = s.totals()
        if ref is None:
            ref = tot
        same = np.array_equal(tot[0], ref[0]) and np.array_equal(tot[1], ref[1])
        if rnd:
            res[i].append(ms)
        print("round %d variant %s: %.4f ms per step, totals %s" % (rnd, v or "default", ms, "same" if same else "DIFFER"), flush=True)
for i, v in enumerate(variants):
    print("%-50s median %.4f ms per step (min %.4f) -> %.3f G reads/s" % (
        v or "default", np.median(res[i]), min(res[i]), a.reads / np.median(res[i]) / 1e6), flush=True)
