#!/usr/bin/env python3
"""Per-kernel timing of index layouts (probe modes) on one data set (development tool; interleaved
rounds in one process, as the CDNA guide's methodology asks). Prints one line per layout."""
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--probes", default="auto", help="index layouts to A/B (SKQ_PROBE values; auto = default)")
ap.add_argument("--pipeline", type=int, default=0, help="also time N batches on two alternating streams")
ap.add_argument("--stamps", action="store_true", help="k_map1 per-wave phase clocks of one launch")
ap.add_argument("--acc-all", action="store_true", help="time every layout with totals accumulated too")
a = ap.parse_args()
ks = [int(x) for x in a.ks.split(",")]
t0 = time.time()
tx = synth.transcriptome(a.ntx, seed=1)
tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
indexes, sessions = {}, {}
for pm in a.probes.split(","):
    # "<kind>/chain": that probe kind plus the chained tables (SKQ_CHAIN=1, the transcripts handed
    # to the index)
    kind, _, part = pm.partition("/")
    if kind == "auto":
        os.environ.pop("SKQ_PROBE", None)
    else:
        os.environ["SKQ_PROBE"] = kind
    os.environ["SKQ_CHAIN"] = "1" if part == "chain" else "0"
    tb = time.time()
    indexes[pm] = skq.Index(ks, tx.ntx, tables, seqs=(tx.seqs, tx.offs) if part == "chain" else None)
    print(pm, indexes[pm].stats(), "built in %.1fs" % (time.time() - tb), flush=True)
os.environ.pop("SKQ_PROBE", None)
os.environ.pop("SKQ_CHAIN", None)
bases, _, _ = synth.reads(tx, a.reads, a.len, seed=1000, err=0.001)
dev = torch.device("cuda", 0)
d = torch.from_numpy(bases).to(dev)
for pm, ix in indexes.items():
    sessions[pm] = skq.Session(ix, a.reads, a.len)
pm0 = a.probes.split(",")[0]
s, index = sessions[pm0], indexes[pm0]
sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
print("setup %.1fs" % (time.time() - t0), flush=True)

def run_layout(sx, acc):
    def f():
        sx.map(d.data_ptr(), None, a.reads, a.len, fixed_len=a.len, stream=sp, accumulate=acc)
    return f


variants = {}
for pm, sx in sessions.items():
    if pm == pm0 or a.acc_all:
        variants[pm + "+acc"] = run_layout(sx, True)
    variants[pm] = run_layout(sx, False)
res = {k: [] for k in variants}
for rnd in range(a.rounds + 1):
    for name, fn in variants.items():
        sx = sessions[name.split("+")[0]]
        sx.enable_timing(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e3
        sx.enable_timing(False)
        k1 = sx.kernel_time(0)[0]
        k2 = sx.kernel_time(1)[0]
        k3 = sx.kernel_time(2)[0]
        k4 = sx.kernel_time(3)[0]
        if rnd:
            res[name].append((wall, k1, k2, k3, k4))
for pm, sx in sessions.items():
    print(pm, "slow reads (sketch, chain) of the last batch:", sx.slow_reads())
# every layout's per-transcript totals over the batch must be identical (each is checked against
# the oracle by the GPU tests; here they are checked against each other at full size)
tot0 = None
for pm, sx in sessions.items():
    sx.reset_totals(sp)
    sx.map(d.data_ptr(), None, a.reads, a.len, fixed_len=a.len, stream=sp, accumulate=True)
    sx.check(sp)
    tot = sx.totals()
    if tot0 is None:
        tot0 = tot
    same = bool(np.array_equal(tot[0], tot0[0]) and np.array_equal(tot[1], tot0[1]))
    print(pm, "totals", "identical to %s" % pm0 if same else "DIFFER from %s" % pm0, int(tot[0].sum()), flush=True)
for name, v in res.items():
    v = np.array(v)
    med = np.median(v, axis=0)
    print("%-10s wall %.3f ms  k_sketch %.3f  k_probe %.3f  k_count %.3f  totals %.3f  -> %.2f G reads/s" % (
        name, med[0], med[1], med[2], med[3], med[4], a.reads / med[0] / 1e6))

if a.pipeline:
    # two sessions on two streams, alternating batches: batch b's chain overlaps batch b+1's
    # sketch (steady-state time per batch of a streamed run)
    s2 = skq.Session(index, a.reads, a.len)
    st = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    ses = [s, s2]
    for acc in (True, False):
        best = 1e9
        for rnd in range(a.rounds + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for b in range(a.pipeline):
                sx, stx = ses[b % 2], st[b % 2]
                sx.map(d.data_ptr(), None, a.reads, a.len, fixed_len=a.len,
                       stream=C.c_void_p(stx.cuda_stream), accumulate=acc)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t) * 1e3 / a.pipeline
            if rnd:
                best = min(best, wall)
        print("pipelined x%d%s: %.3f ms per batch -> %.2f G reads/s" % (
            a.pipeline, " +acc" if acc else "", best, a.reads / best / 1e6))

if a.stamps:
    nw = (a.reads + 255) // 256 * 4
    for v, s in sessions.items():
        buf = torch.zeros(nw * 8, dtype=torch.int64, device=dev)
        s.set_stamps(buf.data_ptr())
        for acc in (True, False):
            s.map(d.data_ptr(), None, a.reads, a.len, fixed_len=a.len, stream=sp, accumulate=acc)
            torch.cuda.synchronize()
            st = buf.view(nw, 8).cpu().numpy().astype(np.int64)
            t0 = st[:, 0].min()
            span = st[:, 5 if acc else 4].max() - t0
            print("stamps %s acc=%d: span %d ticks; per-wave phase ticks (median / mean / p90):" % (v, acc, span))
            names = ["stage", "hash+sort", "gather+insert", "filter+emit", "bin"]
            for i in range(4 + acc):
                dd = st[:, i + 1] - st[:, i]
                print("   %-14s %8.0f %8.0f %8.0f" % (names[i], np.median(dd), dd.mean(), np.percentile(dd, 90)))
            life = st[:, 5 if acc else 4] - st[:, 0]
            print("   %-14s %8.0f %8.0f %8.0f" % ("lifetime", np.median(life), life.mean(), np.percentile(life, 90)))
            # concurrency: waves alive at the median time, and start-time histogram deciles
            starts = st[:, 0] - t0
            print("   start deciles:", [int(x) for x in np.percentile(starts, np.arange(0, 101, 10))])
        s.set_stamps(0)
