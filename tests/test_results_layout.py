"""The device result layouts skq_session_results documents (include/skq.h): the per-wave packed
hashes and candidates of skq_map's fused kernels (layout 1) and the padded rows of skq_sketch +
skq_chain (layout 0), decoded here from the raw device arrays exactly as the header describes and
compared with skq_session_export. The batch includes reads the slow paths take (longer than the
fused kernels' 256 bp, and reads whose k-mers hit more than 16 transcripts), so runs in hash_ext /
cand_ext and their marks are exercised too."""
import ctypes as C

import numpy as np
import pytest
import torch  # noqa: F401  (before skq: one HIP runtime per process)

import skq
from skq import synth

pytestmark = pytest.mark.gpu


def d2h(ptr, dtype, count, at=0):
    out = np.empty(count, dtype)
    if count:
        src = C.c_void_p(ptr + at * np.dtype(dtype).itemsize)
        assert skq.lib().skq_memcpy_d2h(out.ctypes.data_as(C.c_void_p), src, out.nbytes, None) == 0
    return out


def decode(r):
    n, nk, hcap, ccap = r.n_reads, r.nk, r.hcap, r.ccap
    hc = d2h(r.hash_cnt, np.uint32, nk * n).reshape(nk, n)
    cc = d2h(r.cand_cnt, np.uint32, n)
    sets = [[None] * nk for _ in range(n)]
    if r.hash_layout == 1:
        hs = d2h(r.hashes, np.uint32, nk * hcap * n)
        for i in range(nk):
            o = 0
            for q in range(n):
                if q % 64 == 0:
                    o = 0
                c = int(hc[i, q])
                if c & 0x80000000:
                    x = (c & 0xFFFFFF) * 8
                    cnt = int(d2h(r.hash_ext, np.uint32, 1, x)[0])
                    sets[q][i] = d2h(r.hash_ext, np.uint32, cnt, x + 2)
                    o += (c >> 24) & 0x7F
                else:
                    base = i * hcap * n + (q & ~63) * hcap + o
                    sets[q][i] = hs[base:base + c]
                    o += c
    else:
        hs = d2h(r.hashes, np.uint32, nk * hcap * n).reshape(nk, hcap, n)
        for i in range(nk):
            for q in range(n):
                c = int(hc[i, q])
                if c <= hcap:
                    sets[q][i] = hs[i, :c, q]
                else:
                    sets[q][i] = d2h(r.hash_ext, np.uint32, c, int(hs[i, 0, q]))
    cands = []
    if r.cand_layout == 1:
        ct = d2h(r.cand_tid, np.uint32, ccap * n)
        o = 0
        for q in range(n):
            if q % 64 == 0:
                o = 0
            c = int(cc[q])
            if c & 0x80000000:
                x = c & 0x7FFFFFFF
                cnt = int(d2h(r.cand_ext, np.uint32, 1, 2 * x)[0])
                pr = d2h(r.cand_ext, np.uint32, 2 * cnt, 2 * (x + 1)).reshape(-1, 2)
                cands.append((pr[:, 0], pr[:, 1]))
            else:
                w = ct[(q & ~63) * ccap + o:(q & ~63) * ccap + o + c]
                cands.append((w & 0x3FFFFF, w >> 22))
                o += c
    else:
        ct = d2h(r.cand_tid, np.uint32, ccap * n).reshape(ccap, n)
        cs = d2h(r.cand_score, np.uint32, ccap * n).reshape(ccap, n)
        for q in range(n):
            c = int(cc[q])
            if c <= ccap:
                cands.append((ct[:c, q], cs[:c, q]))
            else:
                pr = d2h(r.cand_ext, np.uint32, 2 * c, 2 * int(ct[0, q])).reshape(-1, 2)
                cands.append((pr[:, 0], pr[:, 1]))
    return sets, cands


def batch():
    tx = synth.transcriptome(300, seed=21)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    # 20 copies of one transcript: its reads' k-mers list 20 transcripts (> 16: the slow chain path)
    seqs += [seqs[7]] * 20
    bases, _, _ = synth.reads(tx, 3000, 150, seed=22, err=0.002)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(3000)]
    rng = np.random.default_rng(23)
    for j in rng.choice(3000, 40, replace=False):  # longer than 256 bp: the slow sketch path
        t = int(rng.integers(0, tx.ntx))
        s = tx.seq(t)
        if len(s) > 420:
            a = int(rng.integers(0, len(s) - 400))
            reads[j] = s[a:a + 400]
    seq7 = seqs[7]
    for j in range(100, 160):  # reads of the duplicated transcript
        a = (j * 7) % max(1, len(seq7) - 150)
        reads[j] = seq7[a:a + 150]
    return seqs, reads


@pytest.mark.parametrize("ks", [[31], [21, 31]], ids=["k31", "k21_31"])
@pytest.mark.parametrize("split", [False, True], ids=["map", "sketch+chain"])
def test_results_layout_matches_export(ks, split):
    seqs, reads = batch()
    buf, offs = skq.pack_reads(seqs)
    index = skq.Index(ks, len(seqs), skq.build_tables(buf, offs, ks))
    rb, ro = skq.pack_reads(reads)
    n = len(reads)
    s = skq.Session(index, n, 512)
    d_buf = skq.DeviceBuffer.from_numpy(rb)
    d_offs = skq.DeviceBuffer.from_numpy(ro)
    if split:
        s.sketch(d_buf.ptr, d_offs.ptr, n, 512)
        s.chain(fraction=0.9)
    else:
        s.map(d_buf.ptr, d_offs.ptr, n, 512)
    s.check()
    r = s.results()
    assert r.hash_layout == (0 if split else 1) and r.cand_layout == (0 if split else 1)
    sets, cands = decode(r)
    out = s.export()
    ho, co = out["hash_offs"].astype(np.int64), out["cand_offs"].astype(np.int64)
    nk = len(ks)
    for q in range(n):
        for i in range(nk):
            e = q * nk + i
            np.testing.assert_array_equal(sets[q][i], out["hashes"][ho[e]:ho[e + 1]], err_msg="read %d k %d" % (q, i))
        np.testing.assert_array_equal(cands[q][0], out["cand_tid"][co[q]:co[q + 1]], err_msg="read %d" % q)
        np.testing.assert_array_equal(cands[q][1], out["cand_score"][co[q]:co[q + 1]], err_msg="read %d" % q)
    slow = s.slow_reads()
    assert slow[0] > 0 and slow[1] > 0  # runs were written on both sides
    s.free()
    d_buf.free()
    d_offs.free()
    index.free()


@pytest.mark.parametrize("ks", [[31], [21, 31]], ids=["k31", "k21_31"])
def test_chain_after_map(ks):
    """skq_chain on a fused map's (packed) sketches, at another fraction, equals a map at that
    fraction (which the parity suite pins to the oracle)."""
    seqs, reads = batch()
    buf, offs = skq.pack_reads(seqs)
    index = skq.Index(ks, len(seqs), skq.build_tables(buf, offs, ks))
    rb, ro = skq.pack_reads(reads)
    n = len(reads)
    d_buf = skq.DeviceBuffer.from_numpy(rb)
    d_offs = skq.DeviceBuffer.from_numpy(ro)
    s = skq.Session(index, n, 512)
    s.map(d_buf.ptr, d_offs.ptr, n, 512, fraction=0.9, accumulate=False)
    s.chain(fraction=0.5, accumulate=False)
    s.check()
    a = s.export()
    t = skq.Session(index, n, 512)
    t.map(d_buf.ptr, d_offs.ptr, n, 512, fraction=0.5, accumulate=False)
    t.check()
    b = t.export()
    for key in ("status", "hash_offs", "hashes", "cand_offs", "cand_tid", "cand_score"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)
    for x in (s, t, d_buf, d_offs, index):
        x.free()
