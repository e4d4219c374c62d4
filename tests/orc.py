"""ctypes wrapper over oracle/liboracle.so — TEST INFRASTRUCTURE (the checker, never the product).

Builds the oracle with `make oracle` if the shared object is missing (gcc only, no GPU).
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-C", ROOT, "oracle"], stdout=subprocess.DEVNULL)
        L = C.CDLL(LIB)
        L.orc_seed.restype = C.c_uint64
        L.orc_seed.argtypes = [C.c_ubyte]
        L.orc_srol.restype = C.c_uint64
        L.orc_srol.argtypes = [C.c_uint64]
        L.orc_nthash_fwd.restype = C.c_size_t
        L.orc_nthash_fwd.argtypes = [C.c_char_p, C.c_size_t, C.c_uint, C.c_void_p, C.c_void_p]
        L.orc_threshold.restype = C.c_uint32
        L.orc_threshold.argtypes = [C.c_double]
        L.orc_is_valid_sequence.restype = C.c_int
        L.orc_is_valid_sequence.argtypes = [C.c_char_p, C.c_size_t]
        for fn in (L.orc_sketch,):
            fn.restype = C.c_size_t
            fn.argtypes = [C.c_char_p, C.c_size_t, C.c_uint, C.c_uint32, C.c_void_p]
        L.orc_all_hashes.restype = C.c_size_t
        L.orc_all_hashes.argtypes = [C.c_char_p, C.c_size_t, C.c_uint, C.c_void_p]
        L.orc_index_build.restype = C.c_void_p
        L.orc_index_build.argtypes = [C.c_uint, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32]
        L.orc_index_from_pairs.restype = C.c_void_p
        L.orc_index_from_pairs.argtypes = [C.c_uint, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_index_free.argtypes = [C.c_void_p]
        L.orc_index_nkeys.restype = C.c_uint64
        L.orc_index_nkeys.argtypes = [C.c_void_p, C.c_uint]
        L.orc_index_npost.restype = C.c_uint64
        L.orc_index_npost.argtypes = [C.c_void_p, C.c_uint]
        L.orc_index_export.argtypes = [C.c_void_p, C.c_uint, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_chain_read.restype = C.c_size_t
        L.orc_chain_read.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                                     C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_chain_batch.restype = C.c_int
        L.orc_chain_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_double] + \
                                     [C.c_void_p] * 3 + [C.c_uint64]
        L.orc_map_batch.restype = C.c_int
        L.orc_map_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                    C.c_double] + [C.c_void_p] * 3 + [C.c_uint32] + [C.c_void_p] * 3 + [C.c_uint32]
        L.orc_map_batch_count.restype = C.c_uint64
        L.orc_map_batch_count.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_double]
        L.orc_map_digest.restype = C.c_int
        L.orc_map_digest.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_double, C.c_int,
                                     C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_em.restype = C.c_int
        L.orc_em.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_double,
                             C.c_void_p]
        L.orc_assign.restype = None
        L.orc_assign.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
        L.orc_fastq_map.restype = C.c_int
        L.orc_fastq_map.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_double, C.c_int, C.c_uint64,
                                    C.c_void_p] + [C.c_void_p] * 3 + [C.c_uint32] + [C.c_void_p] * 3 + \
                                   [C.c_uint32] + [C.c_void_p] * 3
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


SKETCH_FRACTION = float(np.float32(0.05))  # src/main.cpp:43 `const float sketch_size = 0.05f`
CHAIN_FRACTION = 0.9                        # src/main.cpp:185


def threshold(fraction=SKETCH_FRACTION):
    return lib().orc_threshold(fraction)


def nthash_fwd(seq: bytes, k: int):
    n = len(seq)
    h = np.zeros(max(n, 1), np.uint64)
    p = np.zeros(max(n, 1), np.uint64)
    m = lib().orc_nthash_fwd(seq, n, k, ptr(h), ptr(p))
    if m == C.c_size_t(-1).value:
        raise ValueError("ntHash argument error")
    return [int(x) for x in h[:m]], [int(x) for x in p[:m]]


def sketch(seq: bytes, k: int, thr=None):
    thr = threshold() if thr is None else thr
    out = np.zeros(max(len(seq), 1), np.uint32)
    m = lib().orc_sketch(seq, len(seq), k, thr, ptr(out))
    if m == C.c_size_t(-1).value:
        raise ValueError("len < k")
    return [int(x) for x in out[:m]]


def all_hashes(seq: bytes, k: int):
    """extract_and_hash_kmers_nthash (src/kmer.cpp:19-35): every window's low 32 bits."""
    out = np.zeros(max(len(seq), 1), np.uint32)
    m = lib().orc_all_hashes(seq, len(seq), k, ptr(out))
    if m == C.c_size_t(-1).value:
        raise ValueError("len < k")
    return [int(x) for x in out[:m]]


class Index:
    """Oracle inverted index (build_kmer_to_transcript_map restated)."""

    def __init__(self, ks, seqs=None, thr=None, pairs=None, ntx=None):
        self.ks = [int(k) for k in ks]
        ka = np.array(self.ks, np.uint32)
        if pairs is not None:
            self.ntx = int(ntx)
            npairs = np.array([len(h) for h, _ in pairs], np.uint64)
            hs = [np.ascontiguousarray(h, np.uint32) for h, _ in pairs]
            ts = [np.ascontiguousarray(t, np.uint32) for _, t in pairs]
            hp = (C.c_void_p * len(hs))(*[x.ctypes.data for x in hs])
            tp = (C.c_void_p * len(ts))(*[x.ctypes.data for x in ts])
            self.h = lib().orc_index_from_pairs(len(self.ks), ptr(ka), self.ntx, ptr(npairs), hp, tp)
        else:
            thr = threshold() if thr is None else thr
            self.ntx = len(seqs)
            buf = b"".join(seqs)
            offs = np.zeros(len(seqs) + 1, np.uint64)
            offs[1:] = np.cumsum([len(s) for s in seqs])
            bb = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
            self.h = lib().orc_index_build(len(self.ks), ptr(ka), self.ntx, ptr(bb), ptr(offs), thr)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_index_free(self.h)
            self.h = None

    def csr(self, i):
        nkeys = lib().orc_index_nkeys(self.h, i)
        npost = lib().orc_index_npost(self.h, i)
        keys = np.zeros(nkeys + 1, np.uint32)
        offs = np.zeros(nkeys + 1, np.uint64)
        tids = np.zeros(npost + 1, np.uint32)
        lib().orc_index_export(self.h, i, ptr(keys), ptr(offs), ptr(tids))
        return keys[:nkeys], offs, tids[:npost]

    def chain(self, sketches, fraction=CHAIN_FRACTION, present=None):
        """orc_chain_read per read: sketches[r][i] = read r's hash set at k slot i (present[r][i]
        False: no sketch at that k). Per read a list of (tid, score), score desc then tid asc."""
        nk = len(self.ks)
        out = []
        cap = max(self.ntx, 1)
        ot = np.zeros(cap, np.uint32)
        os_ = np.zeros(cap, np.uint32)
        for r, sk in enumerate(sketches):
            arrs = [np.ascontiguousarray(np.array(list(sk[i]) or [0], np.uint32)) for i in range(nk)]
            nh = np.array([len(sk[i]) for i in range(nk)], np.uint32)
            pr = np.array([1 if (present is None or present[r][i]) else 0 for i in range(nk)], np.int32)
            hp = (C.c_void_p * nk)(*[a.ctypes.data for a in arrs])
            c = lib().orc_chain_read(self.h, hp, ptr(nh), ptr(pr), fraction, ptr(ot), ptr(os_), cap)
            assert c != C.c_size_t(-1).value
            out.append(list(zip(ot[:c].tolist(), os_[:c].tolist())))
        return out

    def chain_csr(self, hash_offs, hashes, fraction=CHAIN_FRACTION):
        """orc_chain_batch: sketches as CSR (read r, k slot i at hash_offs[r*nk+i]) -> candidates
        (cand_offs[n+1], cand_tid, cand_score), score desc then tid asc."""
        ho = np.ascontiguousarray(hash_offs, np.uint64)
        hs = np.ascontiguousarray(hashes if len(hashes) else np.zeros(1), np.uint32)
        n = (len(ho) - 1) // len(self.ks)
        cap = max(16 * n, 1)
        while True:
            co = np.zeros(n + 1, np.uint64)
            ct = np.zeros(cap, np.uint32)
            cs = np.zeros(cap, np.uint32)
            if lib().orc_chain_batch(self.h, n, ptr(ho), ptr(hs), fraction, ptr(co), ptr(ct), ptr(cs), cap) == 0:
                return co, ct[:co[-1]], cs[:co[-1]]
            cap *= 4

    def map_batch(self, reads, offs=None, thr=None, fraction=CHAIN_FRACTION, hcap=None, ccap=None):
        """reads: list of bytes (or a flat uint8 array + offs). Returns dict of numpy arrays."""
        thr = threshold() if thr is None else thr
        if offs is None:
            buf = np.frombuffer(b"".join(reads) or b"\0", np.uint8)
            offs = np.zeros(len(reads) + 1, np.uint64)
            offs[1:] = np.cumsum([len(r) for r in reads])
        else:
            buf = reads
        n = len(offs) - 1
        nk = len(self.ks)
        maxlen = int(np.max(np.diff(offs))) if n else 1
        hcap = hcap or max(maxlen, 1)
        ccap = ccap or max(self.ntx, 1)
        st = np.zeros(max(n, 1), np.uint8)
        hc = np.zeros(max(n * nk, 1), np.uint32)
        hs = np.zeros(max(n * nk * hcap, 1), np.uint32)
        cc = np.zeros(max(n, 1), np.uint32)
        ct = np.zeros(max(n * ccap, 1), np.uint32)
        cs = np.zeros(max(n * ccap, 1), np.uint32)
        rc = lib().orc_map_batch(self.h, ptr(buf), ptr(offs), n, thr, fraction, ptr(st), ptr(hc),
                                 ptr(hs), hcap, ptr(cc), ptr(ct), ptr(cs), ccap)
        assert rc == 0
        return dict(status=st[:n], hash_cnt=hc[:n * nk].reshape(n, nk),
                    hashes=hs[:n * nk * hcap].reshape(n, nk, hcap), cand_cnt=cc[:n],
                    cand_tid=ct[:n * ccap].reshape(n, ccap), cand_score=cs[:n * ccap].reshape(n, ccap))


def fastq_map(index, fq, nthreads=1, outputs=True, totals=True, hcap=None, ccap=None, thr=None,
              fraction=CHAIN_FRACTION, max_records=None):
    """orc_fastq_map over FASTQ bytes (bytes or a uint8 array): the record machine, per-record
    sketch + chain on nthreads threads, the id map. Returns a dict: n, and when asked the
    per-record outputs (status, hash_cnt, hashes, cand_cnt, cand_tid, cand_score, kept) and the
    per-transcript totals (tx_reads, tx_score)."""
    buf = np.frombuffer(fq, np.uint8) if isinstance(fq, (bytes, bytearray)) else fq
    thr = threshold() if thr is None else thr
    nmax = int(buf.size // 4 + 1) if max_records is None else int(max_records)
    nrec = C.c_uint64()
    nk = len(index.ks)
    res = {}
    if outputs:
        # records are at most one per 4 lines; size the outputs from the line count
        nl = int(np.count_nonzero(buf == 10)) // 4 + 2
        nmax = min(nmax, nl)
        hcap = hcap or 32
        ccap = ccap or max(index.ntx, 1)
        res = dict(status=np.zeros(nmax, np.uint8), hash_cnt=np.zeros(nmax * nk, np.uint32),
                   hashes=np.zeros(nmax * nk * hcap, np.uint32), cand_cnt=np.zeros(nmax, np.uint32),
                   cand_tid=np.zeros(nmax * ccap, np.uint32), cand_score=np.zeros(nmax * ccap, np.uint32),
                   kept=np.zeros(nmax + 1, np.uint8))
    txr = np.zeros(max(index.ntx, 1), np.uint64) if totals else None
    txs = np.zeros(max(index.ntx, 1), np.uint64) if totals else None
    g = lambda k: ptr(res[k]) if outputs else None  # noqa: E731
    rc = lib().orc_fastq_map(index.h, ptr(buf), buf.size, thr, fraction, nthreads, nmax, C.byref(nrec),
                             g("status"), g("hash_cnt"), g("hashes"), hcap or 0, g("cand_cnt"), g("cand_tid"),
                             g("cand_score"), ccap or 0, g("kept"), ptr(txr) if totals else None,
                             ptr(txs) if totals else None)
    if rc != 0:
        raise RuntimeError("orc_fastq_map failed (%d)" % rc)
    n = nrec.value
    out = dict(n=n)
    if outputs:
        out.update(status=res["status"][:n], hash_cnt=res["hash_cnt"][:n * nk].reshape(n, nk),
                   hashes=res["hashes"][:n * nk * hcap].reshape(n, nk, hcap), cand_cnt=res["cand_cnt"][:n],
                   cand_tid=res["cand_tid"][:n * ccap].reshape(n, ccap),
                   cand_score=res["cand_score"][:n * ccap].reshape(n, ccap), kept=res["kept"][:n].astype(bool))
    if totals:
        out.update(tx_reads=txr[:index.ntx], tx_score=txs[:index.ntx])
    return out


def map_digest(index, bases, L, nthreads=1, totals=True, thr=None, fraction=CHAIN_FRACTION):
    """orc_map_digest over fixed-length reads (bases: flat uint8, len n*L): per-read digests
    (tests/digest.py restates them over an skq export) and the per-transcript totals."""
    bases = np.ascontiguousarray(bases, np.uint8)
    n = bases.size // L
    thr = threshold() if thr is None else thr
    dg = np.zeros(max(n, 1), np.uint64)
    txr = np.zeros(max(index.ntx, 1), np.uint64) if totals else None
    txs = np.zeros(max(index.ntx, 1), np.uint64) if totals else None
    rc = lib().orc_map_digest(index.h, ptr(bases), L, n, thr, fraction, nthreads, ptr(dg),
                              ptr(txr) if totals else None, ptr(txs) if totals else None)
    if rc != 0:
        raise RuntimeError("orc_map_digest failed (%d)" % rc)
    out = dict(n=n, digest=dg[:n])
    if totals:
        out.update(tx_reads=txr[:index.ntx], tx_score=txs[:index.ntx])
    return out


def em(cand_offs, cand_tid, cand_score, ntx, max_iterations=20, convergence=0.01):
    """Oracle EM (src/isoform_assignment.cpp:9-65): (pi, iterations)."""
    o = np.ascontiguousarray(cand_offs, np.uint64)
    t = np.ascontiguousarray(cand_tid, np.uint32)
    s = np.ascontiguousarray(cand_score, np.uint32)
    pi = np.zeros(max(ntx, 1), np.float64)
    it = lib().orc_em(len(o) - 1, ptr(o), ptr(t), ptr(s), ntx, max_iterations, convergence, ptr(pi))
    return pi[:ntx], it


def assign(cand_offs, cand_tid, cand_score, ntx, pi):
    o = np.ascontiguousarray(cand_offs, np.uint64)
    t = np.ascontiguousarray(cand_tid, np.uint32)
    s = np.ascontiguousarray(cand_score, np.uint32)
    pi = np.ascontiguousarray(pi, np.float64)
    counts = np.zeros(max(ntx, 1), np.float64)
    assigned = np.zeros(max(ntx, 1), np.uint8)
    lib().orc_assign(len(o) - 1, ptr(o), ptr(t), ptr(s), ntx, ptr(pi), ptr(counts), ptr(assigned))
    return counts[:ntx], assigned[:ntx].astype(bool)
