#!/usr/bin/env python3
"""Same-process A/B of two libskq.so builds (development): each build is loaded as its own copy of
the skq module (ctypes, RTLD_LOCAL: each copy binds to its own kernels), gets its own index and
session over the same tables and the same device-resident reads, and the two are timed in
interleaved rounds, so clock and box drift hit both alike. Also checks that both produce identical
per-transcript totals.

usage: tools/abbench.py LIB_B [--lib-a LIB_A] [--config cfg3] [--rounds 20] [--acc]
       (LIB_A defaults to the product build; e.g. LIB_B = sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so)
"""
import argparse
import ctypes as C
import importlib.util
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sketch-for-rna-seq_amd")
sys.path.insert(0, PKG)
from skq import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib_b")
ap.add_argument("--lib-a", default=os.path.join(PKG, "lib", "libskq.so"))
ap.add_argument("--config", default="cfg3", choices=["cfg2", "cfg3", "cfg5"])
ap.add_argument("--rounds", type=int, default=20)
ap.add_argument("--acc", action="store_true", help="time with the per-transcript totals accumulated")
ap.add_argument("--chain", type=int, default=1, help="SKQ_CHAIN for both indexes")
ap.add_argument("--env-b", default="", help="K=V[,K=V]: environment set only around B's first map (a library "
                "reads its switches once; LIB_B may then be LIB_A itself, loaded as a second copy)")
a = ap.parse_args()
CFG = {"cfg2": (10_000, 1_000_000, 100, [31]), "cfg3": (200_000, 10_000_000, 150, [31]),
       "cfg5": (200_000, 10_000_000, 150, [21, 25, 31])}
ntx, n, L, ks = CFG[a.config]


def load(path, name):
    # (a private copy of the file: dlopen of a path already loaded would return the same library)
    import shutil
    import tempfile
    cp = os.path.join(tempfile.mkdtemp(prefix="skq_ab_"), "libskq.so")
    shutil.copy(path, cp)
    os.environ["SKQ_LIB"] = cp
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, "skq", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.lib()
    return mod


mods = {"A": load(a.lib_a, "skq_a"), "B": load(a.lib_b, "skq_b")}
os.environ["SKQ_CHAIN"] = str(a.chain)
tx = synth.transcriptome(ntx, seed=1)
tables = mods["A"].build_tables(tx.seqs, tx.offs, ks, nthreads=16)
bases, _, _ = synth.reads(tx, n, L, seed=1000, err=0.001)
dev = torch.device("cuda", 0)
d = torch.from_numpy(bases).to(dev)
sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
ix, ss = {}, {}
envb = dict(kv.split("=", 1) for kv in a.env_b.split(",") if kv)
saved = {k_: os.environ.get(k_) for k_ in envb}
for v, m in mods.items():
    for k_, v_ in envb.items():  # (index switches, e.g. SKQ_CHAIN, SKQ_PROBE: read at the build)
        if v == "B":
            os.environ[k_] = v_
        elif saved[k_] is None:
            os.environ.pop(k_, None)
        else:
            os.environ[k_] = saved[k_]
    ix[v] = m.Index(ks, tx.ntx, tables, seqs=(tx.seqs, tx.offs))
    ss[v] = m.Session(ix[v], n, L)
    print(v, {"A": a.lib_a, "B": a.lib_b}[v], ix[v].stats(), flush=True)
res = {v: [] for v in mods}
for rnd in range(a.rounds + 2):
    for v in (("A", "B") if rnd % 2 == 0 else ("B", "A")):
        s = ss[v]
        if True:  # (before every map: some switches are read once, at a copy's first map, others at every map)
            for k_, v_ in envb.items():
                if v == "B":
                    os.environ[k_] = v_
                elif saved[k_] is None:
                    os.environ.pop(k_, None)
                else:
                    os.environ[k_] = saved[k_]
        s.enable_timing(True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.map(d.data_ptr(), None, n, L, fixed_len=L, stream=sp, accumulate=a.acc)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e3
        s.enable_timing(False)
        k = [s.kernel_time(i)[0] for i in range(4)]
        if rnd >= 2:
            res[v].append([wall] + k)
tot = {}
for v, s in ss.items():
    s.reset_totals(sp)
    s.map(d.data_ptr(), None, n, L, fixed_len=L, stream=sp, accumulate=True)
    s.check(sp)
    tot[v] = s.totals()
    print(v, "slow reads (sketch, chain):", s.slow_reads())
same = all(np.array_equal(tot["A"][i], tot["B"][i]) for i in range(2))
print("totals", "IDENTICAL" if same else "DIFFER", flush=True)
for v in mods:
    x = np.array(res[v])
    med = np.median(x, axis=0)
    print("%s  wall %.4f ms  map %.4f ms (min %.4f, p25 %.4f, p75 %.4f)  totals %.4f  -> %.3f G reads/s" % (
        v, med[0], med[1], x[:, 1].min(), np.percentile(x[:, 1], 25), np.percentile(x[:, 1], 75), med[4],
        n / med[0] / 1e6))
ra = np.array(res["A"])[:, 1]
rb = np.array(res["B"])[:, 1]
print("map B/A: median %.4f, paired rounds B/A median %.4f" % (np.median(rb) / np.median(ra), np.median(rb / ra)))
sys.exit(0 if same else 2)
