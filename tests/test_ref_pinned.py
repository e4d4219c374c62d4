"""The oracle (and the product's host IO) pinned against the REFERENCE'S OWN CODE (CPU only).

oracle/_ref/libref.so is /root/reference/src/{sparse_chaining,data_io,isoform_assignment}.cpp
compiled unmodified (oracle/ref.mk) behind a C-ABI harness (oracle/ref_harness.cpp). These tests
close the chain of trust for the legs the ntHash tables cannot pin:

  HIP path == oracle        (tests/test_gpu_parity.py etc., on the GPU, bit-exact)
  oracle   == reference     (here: sparse_chain, EM + assignment, is_valid_sequence)
  product host IO == reference  (here: load_fasta, save_index / load_index both ways, CSV)

The hashing leg (ntHash, a-1/a-2) is pinned by ntHash's own tables (test_oracle_golden.py): the
reference's kmer.cpp / sketch.cpp need the absent ntHash library and are not built.
Skipped when the library cannot be built (no /root/reference, e.g. on the GPU box).
"""
import os
import random
import subprocess

import numpy as np
import pytest

import orc
import refpin
import skq
from skq import synth

pytestmark = pytest.mark.skipif(not refpin.available(), reason="reference sources absent (oracle/_ref not built)")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EDGE = os.path.join(ROOT, "tests", "golden", "edge")
CLI = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "skq")


def _csr(pairs):
    """(hash, tid) pairs -> CSR (keys ascending, offs, tids ascending per key), duplicates removed."""
    h = np.array([p[0] for p in pairs], np.uint32)
    t = np.array([p[1] for p in pairs], np.uint32)
    o = np.lexsort((t, h))
    h, t = h[o], t[o]
    keep = np.ones(len(h), bool)
    keep[1:] = (h[1:] != h[:-1]) | (t[1:] != t[:-1])
    h, t = h[keep], t[keep]
    keys, first = np.unique(h, return_index=True)
    return keys, np.append(first, len(h)).astype(np.uint64), t


def _random_case(seed, ks, index_ks, ntx, nreads, hash_space, maxlist, absent_p=0.0):
    """A random index over index_ks (lists of up to maxlist transcripts over a small hash space,
    so reads hit often and counts tie often) and random read sketches over ks (a mix of index
    keys and misses); some (read, k) sketches absent."""
    rng = random.Random(seed)
    pairs, tables = {}, {}
    for k in index_ks:
        pk = []
        for h in rng.sample(range(hash_space), hash_space // 2):
            for t in rng.sample(range(ntx), rng.randint(1, maxlist)):
                pk.append((h, t))
        pairs[k] = pk
        tables[k] = _csr(pk)
    sketches, present = [], []
    for _ in range(nreads):
        sk, pr = [], []
        for i, k in enumerate(ks):
            if k in ks[:i]:  # a k listed twice: the read has one sketch per k (sketches[k])
                j = ks.index(k)
                sk.append(sk[j])
                pr.append(pr[j])
                continue
            m = rng.choice([0, 1, 2, 3, 5, 8, 13, 21])
            sk.append(set(rng.randrange(hash_space + 50) for _ in range(m)))
            pr.append(rng.random() >= absent_p)
        sketches.append(sk)
        present.append(pr)
    return pairs, tables, sketches, present


def _oracle_index(ks, index_ks, pairs, ntx):
    """The oracle's index over ks: a k missing from the index gets an empty table."""
    return orc.Index(ks, pairs=[([p[0] for p in pairs.get(k, [])], [p[1] for p in pairs.get(k, [])]) for k in ks],
                     ntx=ntx)


@pytest.mark.parametrize("fraction", [0.0, 0.5, 0.9, 1.0, 1.5, -1.0])
@pytest.mark.parametrize("ks,index_ks", [([31], [31]), ([21, 25, 31], [21, 25, 31]),
                                         ([21, 25, 31], [21, 31]),    # k = 25 absent from the index
                                         ([31, 31], [31])])            # a k listed twice
def test_sparse_chain_oracle_equals_reference(fraction, ks, index_ks):
    ntx = 40
    pairs, tables, sketches, present = _random_case(hash((fraction, tuple(ks), tuple(index_ks))) & 0xFFFF, ks,
                                                    index_ks, ntx, 1500, 400, 6, absent_p=0.1)
    ref = refpin.Index(ntx, tables).chain(ks, sketches, fraction, present)
    oi = _oracle_index(ks, index_ks, pairs, ntx)
    got = oi.chain(sketches, fraction, present)
    assert got == ref
    if fraction <= 1.0:
        assert sum(len(c) for c in ref) > 1000  # the case is not vacuous
    else:  # nothing reaches 1.5 x the maximum
        assert sum(len(c) for c in ref) == 0


def test_sparse_chain_ties_and_long_lists():
    """Many transcripts per key and identical counts: the tie order is normalised (score desc,
    tid asc) on both sides; the membership and scores must agree exactly."""
    ntx = 300
    pairs, tables, sketches, _ = _random_case(7, [31], [31], ntx, 800, 60, 40)
    ref = refpin.Index(ntx, tables).chain([31], sketches, 0.9)
    got = _oracle_index([31], [31], pairs, ntx).chain(sketches, 0.9)
    assert got == ref
    assert max(len(c) for c in ref) >= 20


def test_oracle_batch_path_chain_equals_reference():
    """The oracle's whole batch path (records -> sketch -> chain) on synthetic reads: its
    candidates equal the reference's sparse_chain over the oracle's own sketches."""
    tx = synth.transcriptome(400, seed=5)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    ks = [21, 31]
    oi = orc.Index(ks, seqs=seqs)
    tables = {k: oi.csr(i) for i, k in enumerate(ks)}
    bases, _, _ = synth.reads(tx, 3000, 150, seed=6, err=0.003)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(3000)]
    out = oi.map_batch(reads)
    sketches = [[set(out["hashes"][r, i, :out["hash_cnt"][r, i]].tolist()) for i in range(len(ks))]
                for r in range(len(reads))]
    ref = refpin.Index(tx.ntx, tables).chain(ks, sketches, 0.9)
    for r in range(len(reads)):
        c = int(out["cand_cnt"][r])
        assert list(zip(out["cand_tid"][r, :c].tolist(), out["cand_score"][r, :c].tolist())) == ref[r], r
    assert sum(len(c) for c in ref) > 2500


def _random_candidates(rng, nreads, ntx):
    offs, tids, scores = [0], [], []
    for _ in range(nreads):
        c = min(ntx, rng.choice([0, 1, 1, 2, 3, 5, 9]))
        t = rng.sample(range(ntx), c)
        tids += t
        scores += [rng.randint(1, 40) for _ in t]
        offs.append(len(tids))
    return np.array(offs, np.uint64), np.array(tids, np.uint32), np.array(scores, np.uint32)


@pytest.mark.parametrize("nreads,ntx,iters,conv", [(1, 1, 20, 0.01), (50, 7, 20, 0.01), (3000, 400, 20, 0.01),
                                                   (20000, 2000, 100, 0.05), (5000, 300, 3, 0.0)])
def test_em_and_assignment_oracle_and_product_equal_reference(nreads, ntx, iters, conv):
    """estimate_isoform_abundance_em + assign_reads_to_isoforms: the reference adds posteriors in
    unordered_map order, so only a tolerance is meaningful (1e-11 relative)."""
    rng = random.Random(nreads * 31 + ntx)
    o, t, s = _random_candidates(rng, nreads, ntx)
    pi_ref, c_ref, a_ref = refpin.em_assign(o, t, s, ntx, iters, conv)
    pi, it = orc.em(o, t, s, ntx, iters, conv)
    np.testing.assert_allclose(pi, pi_ref, rtol=1e-11, atol=0)
    counts, assigned = orc.assign(o, t, s, ntx, pi)
    np.testing.assert_array_equal(assigned, a_ref)
    np.testing.assert_allclose(counts, c_ref, rtol=1e-11, atol=1e-300)
    # the product's host EM (the drop-in) and assignment
    pi2, it2 = skq.em(o, t, s, ntx, iters, conv, nthreads=4)
    assert it2 == it
    np.testing.assert_allclose(pi2, pi_ref, rtol=1e-11, atol=0)
    c2, a2 = skq.assign(o, t, s, ntx, pi2)
    np.testing.assert_array_equal(a2, a_ref)
    np.testing.assert_allclose(c2, c_ref, rtol=1e-11, atol=1e-300)


def test_is_valid_sequence_equals_reference():
    rng = random.Random(3)
    cases = [b"", b"ACGT", b"acgt", b"ACGN", b"ACG\r", b"AC GT", b"U", b"ACGTU", bytes(range(256))]
    cases += [bytes(rng.choice(b"ACGTNacgt\r ") for _ in range(rng.randint(0, 40))) for _ in range(500)]
    for c in cases:
        assert bool(orc.lib().orc_is_valid_sequence(c, len(c))) == refpin.is_valid_sequence(c), c


def test_load_fasta_equals_reference(tmp_path):
    for path in (os.path.join(EDGE, "e.fa"), _write(tmp_path / "x.fa", b"junk\n>a x y\nAC\n\nGT\n>b\nACGN\n>c\nAC\r\n>d\n")):
        ref = refpin.load_fasta(path, tmp_path)
        names, seqs = skq.fasta_load(path)
        assert dict(zip(names, seqs)) == {i: s for i, (s, _) in ref.items()}
        assert all(ln == 0 for _, ln in ref.values())  # Transcript::length after the move (SURVEY a-8)


def _write(p, b):
    p.write_bytes(b)
    return str(p)


def test_reference_load_index_reads_product_index(tmp_path):
    """skq -o index writes the legacy file; the reference's load_index reads the same content."""
    out = tmp_path / "e.idx"
    subprocess.run([CLI, "-k", "31,25", "-o", "index", os.path.join(EDGE, "e.fa"), str(out)], check=True,
                   capture_output=True, timeout=120)
    ks, tx, maps = refpin.load_index(out, tmp_path)
    pks, names, seqs, tabs = skq.legacy_index_read(out)
    assert ks == pks == [31, 25]
    assert {n: (s, 0) for n, s in zip(names, seqs)} == tx
    for k in (31, 25):
        keys, offs, tids = tabs[k]
        exp = {int(keys[j]): sorted(names[t] for t in tids[offs[j]:offs[j + 1]]) for j in range(len(keys))}
        assert maps[k] == exp


def test_product_reads_reference_saved_index(tmp_path):
    """save_index of the reference -> skq_legacy_index_read: same ks, transcripts, postings."""
    tx = synth.transcriptome(120, seed=9)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    names = [b"ENSTSYN%08d.1|x|" % t for t in range(tx.ntx)]
    ks = [31, 21]
    oi = orc.Index(ks, seqs=seqs)
    tables = {k: oi.csr(i) for i, k in enumerate(ks)}
    p = tmp_path / "ref.idx"
    refpin.save_index(p, ks, names, seqs, tables)
    pks, pnames, pseqs, ptabs = skq.legacy_index_read(p)
    assert pks == ks
    assert dict(zip(pnames, pseqs)) == dict(zip(names, seqs))
    for k in ks:
        keys, offs, tids = tables[k]
        pk, po, pt = ptabs[k]
        np.testing.assert_array_equal(pk, keys)
        np.testing.assert_array_equal(po, offs)
        # tids are dense ids in the file's transcript order: compare by name
        for j in range(len(keys)):
            assert sorted(pnames[x] for x in pt[po[j]:po[j + 1]]) == sorted(names[x] for x in tids[offs[j]:offs[j + 1]])


def test_csv_rows_equal_reference(tmp_path):
    rng = random.Random(4)
    ntx = 500
    o, t, s = _random_candidates(rng, 4000, ntx)
    pi, _ = orc.em(o, t, s, ntx)
    counts, assigned = orc.assign(o, t, s, ntx, pi)
    names = [b"ENSTSYN%08d.1" % i for i in range(ntx)]
    refpin.output_csv(tmp_path / "ref.csv", names, counts, assigned, pi)
    fa = tmp_path / "n.fa"
    fa.write_bytes(b"".join(b">%s\nACGT\n" % n for n in names))
    skq.csv_write(tmp_path / "skq.csv", fa, counts, assigned, pi)
    a = (tmp_path / "ref.csv").read_bytes().split(b"\n")
    b = (tmp_path / "skq.csv").read_bytes().split(b"\n")
    assert a[0] == b[0] == b"Name,NumReads,EM_Abundance"
    assert sorted(x for x in a[1:] if x) == sorted(x for x in b[1:] if x)
    assert len([x for x in a[1:] if x]) == int(assigned.sum()) > 100
