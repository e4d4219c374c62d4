#!/usr/bin/env python3
"""Index build time at the cfg3 transcriptome (200k synthetic transcripts, k=31 and {21,25,31}):
skq_tables_build (host threads) against skq_tables_build_gpu. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import torch  # noqa: E402,F401  (one HIP runtime per process)
import skq  # noqa: E402
from skq import synth  # noqa: E402

tx = synth.transcriptome(200_000, seed=1)
res = {"transcripts": tx.ntx, "bases": int(tx.offs[-1])}
for ks in ([31], [21, 25, 31]):
    skq.build_tables_gpu(tx.seqs, tx.offs, ks)  # warm-up (code objects, allocations)
    t = time.perf_counter()
    g = skq.build_tables_gpu(tx.seqs, tx.offs, ks)
    tg = time.perf_counter() - t
    t = time.perf_counter()
    h = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
    th = time.perf_counter() - t
    same = all((a == b).all() for k in ks for a, b in zip(g[k], h[k]))
    res["k=%s" % ",".join(map(str, ks))] = {"gpu_s": tg, "host16_s": th, "identical": bool(same)}
print(json.dumps(res), flush=True)
