#!/usr/bin/env python3
"""Development check of the chained tables on one GPU: the parity case that failed
(tx300, k = 31, 250 bp), the mismatching reads, and for each the hash whose count differs, with the
host restatement of the read's chain entry (build_chain's rule)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import torch  # noqa: E402,F401
import orc  # noqa: E402
import skq  # noqa: E402
from skq import synth  # noqa: E402

os.environ["SKQ_PROBE"] = "wide"
os.environ["SKQ_CHAIN"] = "1"
L = int(sys.argv[1]) if len(sys.argv) > 1 else 250
tx = synth.transcriptome(300, seed=21)
seqs = [tx.seq(t) for t in range(tx.ntx)]
buf, offs = skq.pack_reads(seqs)
tables = skq.build_tables(buf, offs, [31])
gi = skq.Index([31], len(seqs), tables, seqs=(buf, offs))
print(gi.stats())
oi = orc.Index([31], seqs=seqs)
bases, _, _ = synth.reads(tx, 3000, L, seed=L + 1, err=0.002)
reads = [bases[i * L:(i + 1) * L].tobytes() for i in range(3000)]
rb, ro = skq.pack_reads(reads)
s = skq.Session(gi, 3000, L)
d_b = skq.DeviceBuffer.from_numpy(rb)
d_o = skq.DeviceBuffer.from_numpy(ro)
s.map(d_b.ptr, d_o.ptr, 3000, L)
s.check()
out = s.export()
ref = oi.map_batch(reads)
T = orc.threshold()
keys, koffs, ktids = tables[31]
post = {int(keys[j]): list(ktids[koffs[j]:koffs[j + 1]]) for j in range(len(keys))}
runs = []
for sq in seqs:
    hs, _ = orc.nthash_fwd(sq, 31)
    runs.append([h & 0xFFFFFFFF for h in hs if (h & 0xFFFFFFFF) <= T])
co = out["cand_offs"]
bad = 0
for r in range(3000):
    c = ref["cand_cnt"][r]
    got = list(zip(out["cand_tid"][co[r]:co[r + 1]], out["cand_score"][co[r]:co[r + 1]]))
    exp = list(zip(ref["cand_tid"][r, :c], ref["cand_score"][r, :c]))
    if got == exp:
        continue
    bad += 1
    if bad > 5:
        continue
    hs, _ = orc.nthash_fwd(reads[r], 31)
    rr = [h & 0xFFFFFFFF for h in hs if (h & 0xFFFFFFFF) <= T]
    print("read", r, "got", got, "exp", exp)
    print("  retained (position order):", rr)
    for h in dict.fromkeys(rr):
        print("   ", h, "list", post.get(h))
    q = rr[0]
    succ = {}
    for run in runs:
        for i, h in enumerate(run):
            if h != q:
                continue
            for d in range(1, 9):
                if i + d < len(run) and run[i + d] != h:
                    g = run[i + d]
                    succ[g] = min(succ.get(g, 99), d)
    order = sorted(succ.items(), key=lambda x: (x[1], x[0]))
    slots, ent = 0, []
    for g in [q] + [g for g, _ in order]:
        if g not in post:
            continue
        n = len(post[g])
        need = 2 if 4 <= n <= 7 else 1
        if slots + need > 8:
            break
        slots += need
        ent.append((g, n))
    print("  entry of q =", q, ":", ent)
print("mismatching reads:", bad)
