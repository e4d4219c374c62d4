#!/usr/bin/env python3
"""k_map1 time against the batch size (development tool): one index and session, prefixes of one
device-resident batch, interleaved rounds; prints ms per launch and ms per 1M reads, so the fixed
part (launch ramp, the last round of workgroups) separates from the per-read part.

usage: tools/nsweep.py [--config cfg2] [--ns 250000,500000,1000000,2000000,4000000] [--chain 1]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import skq  # noqa: E402
from skq import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3"])
ap.add_argument("--ns", default="250000,500000,750000,1000000,1280000,1500000,2000000,4000000")
ap.add_argument("--chain", default="1")
ap.add_argument("--rounds", type=int, default=15)
a = ap.parse_args()
ntx, L = {"cfg2": (10_000, 100), "cfg3": (200_000, 150)}[a.config]
ns = [int(x) for x in a.ns.split(",")]
os.environ["SKQ_CHAIN"] = a.chain
tx = synth.transcriptome(ntx, seed=1)
tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=16)
ix = skq.Index([31], tx.ntx, tables, seqs=(tx.seqs, tx.offs))
print(ix.stats(), flush=True)
bases, _, _ = synth.reads(tx, max(ns), L, seed=1000, err=0.001)
d = torch.from_numpy(bases).to("cuda:0")
sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
s = skq.Session(ix, max(ns), L)
res = {n: [] for n in ns}
for rnd in range(a.rounds + 1):
    for n in (ns if rnd % 2 == 0 else ns[::-1]):
        s.enable_timing(True)
        s.map(d.data_ptr(), None, n, L, fixed_len=L, stream=sp, accumulate=True)
        torch.cuda.synchronize()
        s.enable_timing(False)
        if rnd:
            res[n].append(s.kernel_time(0)[0])
for n in ns:
    m = float(np.median(res[n]))
    wg = (n + 255) // 256
    print("n %9d  workgroups %6d (%.2f rounds of 1280)  k_map1 %.4f ms (min %.4f)  %.4f ms per 1M" % (
        n, wg, wg / 1280, m, min(res[n]), m / n * 1e6), flush=True)
