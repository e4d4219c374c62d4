"""The C++ drop-in (include/dropin/*.h: the reference's kmer.h / sketch.h / sparse_chaining.h
signatures over libskq.so), driven by tests/dropin_check.cpp the way src/main.cpp calls it,
checked against the oracle."""
import os
import random
import subprocess

import pytest

import orc
from skq import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "skq_dropin_check")


def test_dropin_driver_is_built():
    assert os.access(BIN, os.X_OK), "run make (build()) first"


@pytest.mark.gpu
def test_dropin_signatures_match_oracle():
    ks = [21, 31]
    tx = synth.transcriptome(120, seed=41)
    names = [n.split("|")[0] for n in tx.names]
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    seqs[-1] = seqs[-1][:150].lower() + b"N" + seqs[-1][151:]  # the unvalidated last record
    bases, _, _ = synth.reads(tx, 400, 150, seed=42)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(400)]
    reads[3] = reads[3][:20]          # too short: dropped by the caller (src/main.cpp:136-138)
    reads[4] = reads[4].lower()       # invalid: dropped (src/main.cpp:132)
    lines = ["K " + ",".join(map(str, ks))]
    lines += ["T %s %s" % (n, s.decode()) for n, s in zip(names, seqs)]
    lines += ["R r%d %s" % (i, r.decode()) for i, r in enumerate(reads)]
    out = subprocess.run([BIN], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True, timeout=300).stdout.splitlines()
    got_s, got_a, got_c, got_v = {}, {}, {}, {}
    for ln in out:
        f = ln.split()
        if f[0] == "S":
            got_s[(f[1], int(f[2]))] = [int(x) for x in f[3:]]
        elif f[0] == "A":
            got_a[(f[1], int(f[2]))] = int(f[3])
        elif f[0] == "V":
            got_v[f[1]] = int(f[2])
        elif f[0] == "C":
            got_c[f[1]] = [(x.rsplit(":", 1)[0], int(x.rsplit(":", 1)[1])) for x in f[2:]]
        elif f[0] == "E":
            assert ln == "E Sequence length is shorter than k-mer length"
    for n, s in zip(names, seqs):
        for k in ks:
            assert got_s[(n, k)] == orc.sketch(s, k), (n, k)
            assert got_a[(n, k)] == len(set(orc.all_hashes(s, k))), (n, k)
    oi = orc.Index(ks, seqs=seqs)
    ref = oi.map_batch(reads)
    for i, r in enumerate(reads):
        rid = "r%d" % i
        assert got_v[rid] == int(all(c in b"ACGT" for c in r))
        if ref["status"][i] != 0:
            assert rid not in got_c
            continue
        c = ref["cand_cnt"][i]
        exp = sorted(((names[t], int(sc)) for t, sc in zip(ref["cand_tid"][i, :c], ref["cand_score"][i, :c])),
                     key=lambda x: (-x[1], x[0]))
        assert got_c[rid] == exp, rid


@pytest.mark.gpu
def test_sketcher_per_call_matches_oracle_and_is_cheap():
    """skq_sketcher_run, the per-sequence path the drop-in's createSketch_FracMinhash_direct and
    extract_and_hash_kmers_nthash take (src/main.cpp:79,143-144 call them once per sequence per
    k): sets equal the oracle's for reads, transcripts, ntHash-skipped bytes, lowercase, U, a k
    longer than the sequence and sequences past the LDS staging size; then the per-call cost on
    150-bp reads (DESIGN.md §2 records it)."""
    import time

    import numpy as np

    import skq

    rng = random.Random(7)
    sk = skq.Sketcher()
    seqs = [bytes(rng.choice(b"ACGT") for _ in range(n)) for n in (31, 32, 100, 150, 151, 999, 5000)]
    seqs.append(b"ACGTNACGTACGTACGTACGTACGTACGTACGTACGTACGTAC" * 5)
    seqs.append(bytes(rng.choice(b"acgtuACGTUN") for _ in range(400)))
    seqs.append(bytes(rng.choice(b"ACGT") for _ in range(60000)))  # (read in place, past the LDS stage)
    seqs.append(b"")
    for s in seqs:
        for k in (21, 25, 31):
            for thr in (None, 0xFFFFFFFF):
                got = set(int(x) for x in sk.run(s, k, thr))
                if len(s) < k:
                    assert got == set()
                    continue
                exp = set(orc.sketch(s, k, thr)) if thr is None else set(orc.all_hashes(s, k))
                assert got == exp, (len(s), k, thr)
    reads = [bytes(rng.choice(b"ACGT") for _ in range(150)) for _ in range(2000)]
    for r in reads[:50]:
        sk.run(r, 31)
    t0 = time.perf_counter()
    for r in reads:
        sk.run(r, 31)
    us = (time.perf_counter() - t0) / len(reads) * 1e6
    print("skq_sketcher_run: %.1f us per 150-bp read (k = 31, %d calls)" % (us, len(reads)))
    assert us < 200.0
    sk.free()
