"""CPU-only tests of the product's host code and the C-ABI library (no GPU calls)."""
import os
import re
import random

import numpy as np
import pytest

import orc
import skq
from skq import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    syms = set()
    for h in ("skq.h", "skq_host.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(skq_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_declared_symbol():
    L = skq.lib()
    declared = _declared_symbols()
    assert len(declared) > 30
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing


def test_threshold_matches_reference_cast():
    assert skq.threshold() == orc.threshold() == 214748367


def test_host_sketch_matches_oracle():
    rng = random.Random(3)
    for trial in range(40):
        k = rng.choice([5, 21, 25, 31, 33, 40])
        s = bytearray(rng.choice(b"ACGTacgtUuNn") for _ in range(rng.randint(k, 600)))
        s = bytes(s)
        assert skq.host_sketch(s, k) == orc.sketch(s, k)
        assert skq.host_sketch(s, k, thr=0xFFFFFFFF) == sorted(set(orc.sketch(s, k, thr=0xFFFFFFFF)))


def _as_pairs(tab):
    keys, offs, tids = tab
    cnt = np.diff(offs.astype(np.int64))
    return np.repeat(keys, cnt), tids


@pytest.mark.parametrize("ks", [[31], [21, 25, 31], [31, 31], [25, 21]])
def test_table_builder_matches_oracle_index(ks):
    tx = synth.transcriptome(300, seed=11)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    # the last FASTA record is unvalidated in the reference: give some transcripts N / lowercase
    seqs[5] = seqs[5][:100] + b"N" + seqs[5][101:]
    seqs[6] = seqs[6].lower()
    seqs[7] = seqs[7][:20]  # shorter than every k: not indexed
    buf, offs = skq.pack_reads(seqs)
    got = skq.build_tables(buf, offs, ks, nthreads=4)
    oi = orc.Index(ks, seqs=seqs)
    assert sorted(got) == sorted(set(ks))
    for i, k in enumerate(ks):
        ok, oo, ot = oi.csr(i)
        gk, go, gt = got[k]
        np.testing.assert_array_equal(gk, ok)
        np.testing.assert_array_equal(go, oo)
        np.testing.assert_array_equal(gt, ot)
    assert 7 not in set(got[ks[0]][2].tolist())


def test_synth_is_deterministic():
    a = synth.transcriptome(50, seed=5)
    b = synth.transcriptome(50, seed=5)
    assert a.names == b.names and np.array_equal(a.seqs, b.seqs)
    r1, t1, s1 = synth.reads(a, 100, 150, seed=9)
    r2, t2, s2 = synth.reads(b, 100, 150, seed=9)
    assert np.array_equal(r1, r2) and np.array_equal(t1, t2)
    # reads come from their transcript (up to the substitution rate)
    same = 0
    for r in range(100):
        same += r1[r * 150:(r + 1) * 150].tobytes() == a.seq(t1[r])[s1[r]:s1[r] + 150]
    assert same > 80
