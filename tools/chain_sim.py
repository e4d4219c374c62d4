#!/usr/bin/env python3
"""CPU estimate for chained index entries: how many random index requests a read
needs when each key's 128-B entry also carries the postings lists of the keys that FOLLOW it along
the transcripts (its successors within H retained k-mers), so that one request can settle several
of a read's retained hashes. A read covers a contiguous run of a transcript's retained k-mers, so
the entry of its first one usually holds the rest.

usage: tools/chain_sim.py [--ntx 20000] [--reads 50000] [--k 31] [--hops 1,2,4,6,8] [--words 32]
Prints mean requests per read (k_map1 today: one per retained hash).
"""
import argparse
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import orc  # noqa: E402  (the oracle's ntHash, CPU)
from skq import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ntx", type=int, default=20000)
ap.add_argument("--reads", type=int, default=50000)
ap.add_argument("--len", type=int, default=150)
ap.add_argument("--k", type=int, default=31)
ap.add_argument("--hops", default="1,2,4,6,8,12")
ap.add_argument("--words", default="16,32,64")
ap.add_argument("--both", action="store_true", help="neighbours on both sides; queries in value order")
ap.add_argument("--single", action="store_true", help="word layout, one chain request per read, the rest one each")
ap.add_argument("--slots", type=int, default=0, help="slot layout: N slots of 4 words (a list of <= 3 tids takes one "
                "slot, 4-7 two, longer one); one chain request per read, the rest one request per hash")
a = ap.parse_args()
T = orc.threshold()


def retained_in_order(s):
    hs, pos = orc.nthash_fwd(s, a.k)
    return [h & 0xFFFFFFFF for h in hs if (h & 0xFFFFFFFF) <= T]


tx = synth.transcriptome(a.ntx, seed=1)
runs = [retained_in_order(tx.seq(t)) for t in range(tx.ntx)]
post = collections.defaultdict(set)
for t, r in enumerate(runs):
    for h in r:
        post[h].add(t)
print("keys %d, mean list %.2f" % (len(post), np.mean([len(v) for v in post.values()])))
bases, _, _ = synth.reads(tx, a.reads, a.len, seed=3, err=0.001)
rr = [retained_in_order(bases[i * a.len:(i + 1) * a.len].tobytes()) for i in range(a.reads)]
print("retained per read %.2f (distinct %.2f)" % (np.mean([len(r) for r in rr]), np.mean([len(set(r)) for r in rr])))


def rec_words(h):
    n = len(post[h])
    if a.slots:
        return 1 if (n <= 3 or n > 7) else 2
    return 1 + (n if n <= 7 else 1)


for H in [int(x) for x in a.hops.split(",")]:
    # successors within H retained positions, nearest first (by the smallest hop seen)
    succ = collections.defaultdict(dict)
    for r in runs:
        for i, h in enumerate(r):
            for d in range(1, H + 1):
                for j in ((i + d, i - d) if a.both else (i + d,)):
                    if j < 0 or j >= len(r):
                        continue
                    g = r[j]
                    if g != h and (g not in succ[h] or succ[h][g] > d):
                        succ[h][g] = d
    for W in ([a.slots] if a.slots else [int(x) for x in a.words.split(",")]):
        cover = {}
        full = 0
        for h in post:
            used = rec_words(h)
            c = {h}
            for g, d in sorted(succ[h].items(), key=lambda x: x[1]):
                w = rec_words(g)
                if used + w > W:
                    full += 1
                    break
                used += w
                c.add(g)
            cover[h] = c
        req = []
        for r in rr:
            left = set(r)
            n = 0
            if a.slots or a.single:  # one chain request (the first retained hash), then one per uncovered hash
                if r:
                    left -= cover.get(r[0], {r[0]})
                    left.discard(r[0])
                    n = 1 + len(left)
                req.append(n)
                continue
            for h in (sorted(set(r)) if a.both else r):  # position order (value order with --both)
                if h not in left:
                    continue
                n += 1
                left -= cover.get(h, {h})
                left.discard(h)
            req.append(n)
        print("hops %2d, entry %3d words: %.3f requests per read (%.1f %% of the hashes), %.1f %% of entries full" % (
            H, W, np.mean(req), 100.0 * np.mean(req) / np.mean([len(set(r)) for r in rr]), 100.0 * full / len(post)),
            flush=True)
