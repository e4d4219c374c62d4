#!/usr/bin/env python3
"""CPU estimate (development): how many of a read's retained hashes its chained entry settles when
the records are matched by position instead of against every hash of the read.

The entries follow build_chain / chain_entry (skq_capi.hip): the key's own record, then successor
keys within CHAIN_HOPS retained positions along any transcript, nearest first (ties: smaller key),
while they fit 16 records over 8 distinct transcripts. A read's query is its first retained
window (position order). Matching rules compared:
  any      every record against every retained hash of the read (k_map1, round 4);
  off+-t   record g, first seen at hop o, against the read's retained windows o-t..o+t only.
Prints, per rule, the mean distinct hashes per read left for the wide entries.

usage: tools/chain_offsets_sim.py [--ntx 20000] [--reads 40000]
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
ap.add_argument("--reads", type=int, default=40000)
ap.add_argument("--len", type=int, default=150)
ap.add_argument("--k", type=int, default=31)
ap.add_argument("--err", type=float, default=0.001)
a = ap.parse_args()
T = orc.threshold()
HOPS, KEYS, TIDS = 12, 16, 8


def retained_in_order(s):
    hs, _ = orc.nthash_fwd(s, a.k)
    return [h & 0xFFFFFFFF for h in hs if (h & 0xFFFFFFFF) <= T]


tx = synth.transcriptome(a.ntx, seed=1)
runs = [retained_in_order(tx.seq(t)) for t in range(tx.ntx)]
post = collections.defaultdict(set)
for t, r in enumerate(runs):
    for h in r:
        post[h].add(t)
cand = collections.defaultdict(dict)  # key -> successor -> smallest hop
for r in runs:
    for i, h in enumerate(r):
        for d in range(1, HOPS + 1):
            if i + d >= len(r):
                break
            g = r[i + d]
            if g != h and (g not in cand[h] or cand[h][g] > d):
                cand[h][g] = d
entry = {}
for h in post:
    if len(post[h]) > TIDS:
        entry[h] = {}
        continue
    tids = set(post[h])
    recs = {h: 0}
    for g, d in sorted(cand[h].items(), key=lambda x: (x[1], x[0])):
        if len(recs) == KEYS:
            break
        if len(post[g]) > TIDS or len(tids | post[g]) > TIDS:
            continue
        tids |= post[g]
        recs[g] = d
    entry[h] = recs
bases, _, _ = synth.reads(tx, a.reads, a.len, seed=3, err=a.err)
rr = [retained_in_order(bases[i * a.len:(i + 1) * a.len].tobytes()) for i in range(a.reads)]
nd = np.mean([len(set(r)) for r in rr])
print("transcripts %d, keys %d, reads %d: %.2f retained windows, %.2f distinct per read" % (
    a.ntx, len(post), a.reads, np.mean([len(r) for r in rr]), nd))
for rule in ["any", 0, 1, 2]:
    left = []
    for r in rr:
        if not r:
            left.append(0)
            continue
        recs = entry.get(r[0], {})
        if rule == "any":
            settled = set(r) & set(recs)
        else:
            settled = set()
            for g, o in recs.items():
                for j in range(max(0, o - rule), min(len(r), o + rule + 1)):
                    if r[j] == g:
                        settled.add(g)
                        break
        left.append(len(set(r) - settled))
    print("  %-6s %.3f distinct hashes per read to the wide entries (%.1f %%)" % (
        rule if rule == "any" else "off+-%d" % rule, np.mean(left), 100 * np.mean(left) / nd), flush=True)
