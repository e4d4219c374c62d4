#!/usr/bin/env python3
"""CPU-baseline calibration: the reference's OWN sparse_chain
(src/sparse_chaining.cpp:29-115, compiled unmodified into oracle/_ref/libref.so) against the oracle's
chain (oracle/oracle.c orc_chain_batch) on identical sketches, one core each, at cfg3's shape
(200k synthetic transcripts, 150 bp reads, k = 31, sketch fraction (double)0.05f, chain 0.9).

Runs in the BUILD container only (it needs /root/reference); writes profiles/cpu_calibration.json,
whose "summary" bench.py copies into cpu_baseline.calibration. The candidate lists of the two are
compared as well (another pin of the oracle's chain at full index scale).

The reference's sketch leg (kmer.cpp / sketch.cpp) needs the absent ntHash library and is not
built, so only the chain leg is calibrated; the sketch leg's timing comes from the oracle alone.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import orc  # noqa: E402
import refpin  # noqa: E402
from skq import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntx", type=int, default=200_000)
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_calibration.json"))
    a = ap.parse_args()
    assert refpin.available(), "oracle/_ref/libref.so missing (needs /root/reference)"
    L, n, k = a.read_len, a.reads, 31

    t0 = time.time()
    tx = synth.transcriptome(a.ntx, seed=1)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    oi = orc.Index([k], seqs=seqs)
    keys, offs, tids = oi.csr(0)
    print("index: %d transcripts, %d keys, %d postings (%.1fs)" % (tx.ntx, len(keys), len(tids), time.time() - t0),
          flush=True)
    t0 = time.time()
    ri = refpin.Index(tx.ntx, {k: (keys, offs, tids)})
    print("reference kmer_to_transcripts built (%.1fs)" % (time.time() - t0), flush=True)

    bases, _, _ = synth.reads(tx, n, L, seed=1000, err=0.001)
    ro = np.arange(n + 1, dtype=np.uint64) * L
    tc = time.perf_counter()
    mb = orc.Index.map_batch(oi, bases, offs=ro, hcap=64, ccap=64)
    t_map = time.perf_counter() - tc
    hc = mb["hash_cnt"][:, 0].astype(np.int64)
    ho = np.zeros(n + 1, np.uint64)
    ho[1:] = np.cumsum(hc)
    hs = mb["hashes"][:, 0, :][np.arange(64)[None, :] < hc[:, None]]

    tc = time.perf_counter()
    oc = oi.chain_csr(ho, hs)
    t_orc = time.perf_counter() - tc
    rc = ri.chain_csr([k], ho, hs)
    t_ref = rc[3]
    same = all(np.array_equal(x, y) for x, y in zip(oc, rc[:3]))
    summary = {
        "what": "reference sparse_chain (compiled unmodified, g++ -O2) vs oracle orc_chain_batch on identical "
                "sketches, 1 core each, in the build container",
        "shape": "%d synthetic transcripts, %d reads x %d bp, k=%d, fraction (double)0.05f, chain 0.9"
                 % (tx.ntx, n, L, k),
        "reference_chain_reads_per_s": n / t_ref,
        "oracle_chain_reads_per_s": n / t_orc,
        "oracle_over_reference": t_ref / t_orc,
        "oracle_sketch_plus_chain_reads_per_s": n / t_map,
        "candidate_lists_identical": bool(same),
        "note": "reference sketch leg (ntHash) unbuildable here; the oracle's sketch + chain rate is given beside "
                "the reference chain rate; the survey measured the reference CPU hot path (shim ntHash build) at "
                "105k reads/s on 1 core at cfg3 (SURVEY.md §6)",
    }
    res = {"summary": summary, "candidates": int(oc[0][-1]), "retained_hashes": int(ho[-1]),
           "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t")}
    print(json.dumps(res, indent=1))
    if not same:
        raise SystemExit("candidate lists differ between the reference and the oracle")
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
