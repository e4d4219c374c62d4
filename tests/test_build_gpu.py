"""Index building on the GPU (skq_tables_build_gpu) against the host builder (skq_tables_build)
and the oracle's transcript sketches: identical CSR tables, bit for bit."""
import os
import random
import subprocess

import numpy as np
import pytest

import orc
import skq
from skq import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "skq")


def same(a, b):
    assert set(a) == set(b)
    for k in a:
        for x, y in zip(a[k], b[k]):
            np.testing.assert_array_equal(x, y)


def odd_transcripts(seed=3, n=400):
    """Synthetic transcripts with the bytes ntHash treats specially: lowercase, U/u, N and other
    bytes (windows skipped), short ones (left out), one of exactly the largest k."""
    tx = synth.transcriptome(n, seed=seed)
    rng = random.Random(seed)
    seqs = []
    for t in range(tx.ntx):
        s = bytearray(tx.seq(t))
        for _ in range(rng.randint(0, 4)):
            i = rng.randrange(len(s))
            s[i] = rng.choice(b"NnRx-acgtuU")
        if rng.random() < 0.1:
            s = s.lower()
        seqs.append(bytes(s))
    seqs += [b"ACGT" * 5, b"A" * 31, b"ACGU" * 40, b"", b"N" * 100]
    return seqs


@pytest.mark.parametrize("ks", [[31], [21, 25, 31], [31, 31], [19, 25]])
def test_gpu_tables_equal_host_tables(ks):
    seqs = odd_transcripts()
    buf, offs = skq.pack_reads(seqs)
    same(skq.build_tables_gpu(buf, offs, ks), skq.build_tables(buf, offs, ks))


def test_gpu_tables_equal_the_oracle():
    seqs = odd_transcripts(seed=8, n=150)
    buf, offs = skq.pack_reads(seqs)
    ks = [21, 31]
    got = skq.build_tables_gpu(buf, offs, ks)
    oi = orc.Index(ks, seqs=seqs)
    for i, k in enumerate(ks):
        for a, b in zip(got[k], oi.csr(i)):
            np.testing.assert_array_equal(a, b)


def test_gpu_tables_at_scale():
    tx = synth.transcriptome(20_000, seed=5)
    same(skq.build_tables_gpu(tx.seqs, tx.offs, [31]), skq.build_tables(tx.seqs, tx.offs, [31]))


def test_gpu_tables_threshold_above_the_capacity_guess():
    """Every window retained (threshold UINT32_MAX): the first pass overflows its 6 % guess and
    the builder re-runs with the exact count."""
    seqs = odd_transcripts(seed=4, n=60)
    buf, offs = skq.pack_reads(seqs)
    same(skq.build_tables_gpu(buf, offs, [25], thr=0xFFFFFFFF), skq.build_tables(buf, offs, [25], thr=0xFFFFFFFF))


def test_cli_index_on_the_gpu(tmp_path):
    edge = os.path.join(ROOT, "tests", "golden", "edge", "e.fa")
    out = tmp_path / "g.idx"
    subprocess.run([CLI, "-k", "31,25", "-o", "index", edge, str(out)], check=True, capture_output=True,
                   timeout=120)
    ks, names, seqs, tabs = skq.legacy_index_read(out)
    buf, offs = skq.pack_reads(seqs)
    same(tabs, skq.build_tables(buf, offs, [31, 25]))


def test_chained_host_build_shared_between_concurrent_indexes():
    """Indexes built at once from the same tables and sequences (the CLI's one thread per device)
    share one host build of the chained entries: one reports the build's seconds, the other 0, and
    both map a batch identically (the share was keyed on a per-call vector's
    address, so it never happened)."""
    import threading
    tx = synth.transcriptome(200_000, seed=1)
    tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=16)
    out, errs = [None, None], []
    go = threading.Barrier(2)

    def make(i):
        try:
            go.wait()
            out[i] = skq.Index([31], tx.ntx, tables, seqs=(tx.seqs, tx.offs))
        except Exception as ex:  # noqa: BLE001
            errs.append(ex)

    th = [threading.Thread(target=make, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    st = [ix.stats() for ix in out]
    assert all(s["chained"] > 2 for s in st), st
    secs = sorted(s["chain_build_s"] for s in st)
    assert secs[0] == 0 and secs[1] > 0, st
    bases, _, _ = synth.reads(tx, 20_000, 150, seed=9)
    d = skq.DeviceBuffer.from_numpy(bases)
    res = []
    for ix in out:
        s = skq.Session(ix, 20_000, 150)
        s.map(d.ptr, None, 20_000, 150, fixed_len=150)
        s.check()
        e = s.export()
        res.append((e["cand_offs"], e["cand_tid"], e["cand_score"], e["hashes"]))
        s.free()
        ix.free()
    d.free()
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)
