"""ctypes wrapper over oracle/_ref/libref.so — the reference's OWN sparse_chain, EM, assignment,
is_valid_sequence, load_fasta, save_index / load_index and output_to_csv, compiled unmodified from
/root/reference/src (oracle/ref.mk) behind oracle/ref_harness.cpp. TEST INFRASTRUCTURE: it pins
the oracle (and the product's host IO) against the reference; nothing in the product loads it.

available() is False when the library is absent and cannot be built (no /root/reference, e.g. on
the GPU box); the tests that need it skip then.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libref.so")
REF = "/root/reference"

_lib = None


def available():
    if not os.path.exists(LIB) and os.path.isdir(REF):
        subprocess.run(["make", "-C", ROOT, "-f", "oracle/ref.mk"], stdout=subprocess.DEVNULL, check=False)
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        L.ref_index_new.restype = vp
        L.ref_index_new.argtypes = [u32, vp, C.c_uint, vp, vp, vp, vp, vp]
        L.ref_index_free.argtypes = [vp]
        L.ref_chain.restype = C.c_int
        L.ref_chain.argtypes = [vp, u64, C.c_uint, vp, vp, vp, vp, C.c_double, vp, vp, vp, u64]
        L.ref_chain_seconds.restype = C.c_double
        L.ref_chain_seconds.argtypes = []
        L.ref_em_assign.restype = None
        L.ref_em_assign.argtypes = [u64, vp, vp, vp, u32, C.c_int, C.c_double, vp, vp, vp]
        L.ref_output_csv.restype = C.c_int
        L.ref_output_csv.argtypes = [C.c_char_p, u32, vp, vp, vp, vp]
        L.ref_is_valid_sequence.restype = C.c_int
        L.ref_is_valid_sequence.argtypes = [C.c_char_p, u64]
        L.ref_load_fasta_dump.restype = C.c_int
        L.ref_load_fasta_dump.argtypes = [C.c_char_p, C.c_char_p]
        L.ref_save_index.restype = C.c_int
        L.ref_save_index.argtypes = [C.c_char_p, C.c_uint, vp, u32, vp, vp, vp, vp, vp, vp, vp]
        L.ref_load_index_dump.restype = C.c_int
        L.ref_load_index_dump.argtypes = [C.c_char_p, C.c_char_p]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _names(names):
    arr = (C.c_char_p * len(names))(*[bytes(n) for n in names])
    return arr


class _Tables:
    """Per-k CSR arrays kept alive for a call: (ks, nkeys, key/off/tid pointer arrays)."""

    def __init__(self, ks, tables):
        self.ks = np.array(ks, np.uint32)
        self.keep = []
        keys, offs, tids, nkeys = [], [], [], []
        for k in ks:
            kk, oo, tt = tables[k]
            kk = np.ascontiguousarray(kk, np.uint32)
            oo = np.ascontiguousarray(oo, np.uint64)
            tt = np.ascontiguousarray(tt if len(tt) else np.zeros(1, np.uint32), np.uint32)
            if not len(kk):
                kk = np.zeros(1, np.uint32)
            self.keep += [kk, oo, tt]
            keys.append(kk.ctypes.data)
            offs.append(oo.ctypes.data)
            tids.append(tt.ctypes.data)
            nkeys.append(len(tables[k][0]))
        self.nkeys = np.array(nkeys, np.uint64)
        self.keys = (C.c_void_p * len(ks))(*keys)
        self.offs = (C.c_void_p * len(ks))(*offs)
        self.tids = (C.c_void_p * len(ks))(*tids)


class Index:
    """The reference's kmer_to_transcripts built from CSR tables {k: (keys, offs, tids)}."""

    def __init__(self, ntx, tables, names=None):
        self.ntx = ntx
        ks = sorted(tables)
        t = _Tables(ks, tables)
        nm = _names(names) if names is not None else None
        self.h = lib().ref_index_new(ntx, C.cast(nm, C.c_void_p) if nm is not None else None, len(ks), _p(t.ks),
                                     _p(t.nkeys), t.keys, t.offs, t.tids)

    def chain(self, ks, sketches, fraction=0.9, present=None):
        """sparse_chain over reads' sketches: sketches[r][i] = the hash set of read r at ks[i]
        (present[r][i] False: that k is absent from the read's MultiKmerSketch). Returns per read
        a list of (tid, score), score desc then tid asc."""
        n, nk = len(sketches), len(ks)
        ho = np.zeros(n * nk + 1, np.uint64)
        flat = []
        for r in range(n):
            for i in range(nk):
                flat.extend(int(x) for x in sketches[r][i])
                ho[r * nk + i + 1] = len(flat)
        hs = np.array(flat or [0], np.uint32)
        pr = None
        if present is not None:
            pr = np.array([[1 if present[r][i] else 0 for i in range(nk)] for r in range(n)], np.uint8).reshape(-1)
            if not len(pr):
                pr = np.zeros(1, np.uint8)
        cap = max(1, 16 * n)
        ka = np.array(ks, np.uint32)
        while True:  # -1: more candidates than cap
            co = np.zeros(n + 1, np.uint64)
            ct = np.zeros(cap, np.uint32)
            cs = np.zeros(cap, np.uint32)
            rc = lib().ref_chain(self.h, n, nk, _p(ka), _p(ho), _p(hs), _p(pr) if pr is not None else None,
                                 fraction, _p(co), _p(ct), _p(cs), cap)
            if rc == 0:
                break
            cap *= 4
        return [list(zip(ct[co[r]:co[r + 1]].tolist(), cs[co[r]:co[r + 1]].tolist())) for r in range(n)]

    def chain_csr(self, ks, hash_offs, hashes, fraction=0.9):
        """sparse_chain over sketches given as CSR (read r, k slot i at hash_offs[r*nk+i]), every k
        present. Returns (cand_offs, cand_tid, cand_score, seconds inside sparse_chain itself)."""
        ho = np.ascontiguousarray(hash_offs, np.uint64)
        hs = np.ascontiguousarray(hashes if len(hashes) else np.zeros(1), np.uint32)
        ka = np.array(ks, np.uint32)
        n = (len(ho) - 1) // len(ks)
        cap = max(16 * n, 1)
        while True:
            co = np.zeros(n + 1, np.uint64)
            ct = np.zeros(cap, np.uint32)
            cs = np.zeros(cap, np.uint32)
            if lib().ref_chain(self.h, n, len(ks), _p(ka), _p(ho), _p(hs), None, fraction, _p(co), _p(ct), _p(cs),
                               cap) == 0:
                return co, ct[:co[-1]], cs[:co[-1]], lib().ref_chain_seconds()
            cap *= 4

    def __del__(self):
        if getattr(self, "h", None):
            lib().ref_index_free(self.h)
            self.h = None


def em_assign(cand_offs, cand_tid, cand_score, ntx, max_iterations=20, convergence=0.01):
    """estimate_isoform_abundance_em + assign_reads_to_isoforms: (pi, counts, assigned)."""
    o = np.ascontiguousarray(cand_offs, np.uint64)
    t = np.ascontiguousarray(cand_tid if len(cand_tid) else np.zeros(1), np.uint32)
    s = np.ascontiguousarray(cand_score if len(cand_score) else np.zeros(1), np.uint32)
    pi = np.zeros(max(ntx, 1))
    counts = np.zeros(max(ntx, 1))
    assigned = np.zeros(max(ntx, 1), np.uint8)
    lib().ref_em_assign(len(o) - 1, _p(o), _p(t), _p(s), ntx, max_iterations, convergence, _p(pi), _p(counts),
                        _p(assigned))
    return pi[:ntx], counts[:ntx], assigned[:ntx].astype(bool)


def output_csv(path, names, counts, assigned, pi):
    nm = _names(names)
    c = np.ascontiguousarray(counts, np.float64)
    a = np.ascontiguousarray(assigned, np.uint8)
    p = np.ascontiguousarray(pi, np.float64)
    assert lib().ref_output_csv(str(path).encode(), len(names), C.cast(nm, C.c_void_p), _p(c), _p(a), _p(p)) == 0


def is_valid_sequence(seq: bytes):
    return bool(lib().ref_is_valid_sequence(seq, len(seq)))


def load_fasta(path, tmp):
    """load_fasta: {id: (sequence, length)}."""
    out = os.path.join(str(tmp), "fasta.dump")
    assert lib().ref_load_fasta_dump(str(path).encode(), out.encode()) == 0
    res = {}
    for line in open(out, "rb").read().split(b"\n"):
        if line:
            i, s, ln = line.split(b"\t")
            res[i] = (s, int(ln))
    return res


def save_index(path, ks, names, seqs, tables):
    t = _Tables(ks, tables)
    nm = _names(names)
    buf = np.frombuffer(b"".join(seqs) or b"\0", np.uint8)
    so = np.zeros(len(seqs) + 1, np.uint64)
    so[1:] = np.cumsum([len(s) for s in seqs])
    assert lib().ref_save_index(str(path).encode(), len(ks), _p(t.ks), len(names), C.cast(nm, C.c_void_p), _p(buf),
                                _p(so), _p(t.nkeys), t.keys, t.offs, t.tids) == 0


def load_index(path, tmp):
    """load_index, canonical: (ks in file order, {id: (seq, length)}, {k: {key: sorted ids}})."""
    out = os.path.join(str(tmp), "index.dump")
    assert lib().ref_load_index_dump(str(path).encode(), out.encode()) == 0
    ks, tx, maps = [], {}, {}
    for line in open(out, "rb").read().split(b"\n"):
        if line.startswith(b"K"):
            ks = [int(x) for x in line.split()[1:]]
        elif line.startswith(b"T "):
            i, s, ln = line[2:].split(b"\t")
            tx[i] = (s, int(ln))
        elif line.startswith(b"M "):
            f = line.split(b" ")
            maps.setdefault(int(f[1]), {})[int(f[2])] = f[3:]
    return ks, tx, maps
