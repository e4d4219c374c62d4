"""Python binding (ctypes) over the C ABI in include/skq.h — for tests, bench.py and scripting.

The hot path is the HIP code in libskq.so; this module only moves arrays across the boundary.
Loading fails loudly when the shared library is missing: there is no CPU fallback.

If PyTorch is used in the same process, import torch BEFORE this module so that torch's HIP
runtime is the one libskq.so binds to (same SONAME, one runtime per process).
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SKQ_LIB") or os.path.join(PKG_DIR, "lib", "libskq.so")  # SKQ_LIB: dev builds

SKQ_MAX_K = 8
READ_OK, READ_INVALID, READ_SHORT = 0, 1, 2

_lib = None


class SkqError(RuntimeError):
    pass


class _KmerTable(C.Structure):
    _fields_ = [("k", C.c_uint32), ("nkeys", C.c_uint64), ("keys", C.c_void_p), ("offs", C.c_void_p),
                ("tids", C.c_void_p)]


class _Results(C.Structure):
    _fields_ = [("n_reads", C.c_uint64), ("nk", C.c_uint32), ("hcap", C.c_uint32), ("ccap", C.c_uint32),
                ("ntx", C.c_uint32)] + [(n, C.c_void_p) for n in (
                    "status", "hash_cnt", "hashes", "hash_ext", "cand_cnt", "cand_tid", "cand_score",
                    "cand_ext", "tx_reads", "tx_score")] + [("hash_layout", C.c_uint32),
                                                               ("cand_layout", C.c_uint32)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SkqError("libskq.so not built (%s): run `make` or __graft_entry__.build()" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        vp, u32, u64, i32, dbl = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_double
        sig = {
            "skq_last_error": (C.c_char_p, []),
            "skq_version": (i32, []),
            "skq_device_count": (i32, []),
            "skq_threshold": (u32, [dbl]),
            "skq_index_create": (i32, [i32, u32, u32, vp, u32, vp, C.POINTER(vp)]),
            "skq_index_free": (i32, [vp]),
            "skq_index_stats": (i32, [vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u32)]),
            "skq_index_direct": (i32, [vp]),
            "skq_index_chained": (C.c_double, [vp]),
            "skq_index_chain_build": (i32, [vp, C.POINTER(C.c_double), C.POINTER(u64)]),
            "skq_index_create_chained": (i32, [i32, u32, u32, vp, u32, vp, vp, vp, u32, u32, C.POINTER(vp)]),
            "skq_session_slow_reads": (i32, [vp, C.POINTER(u32), C.POINTER(u32)]),
            "skq_session_slow_counts": (i32, [vp, C.POINTER(u32)]),
            "skq_session_create": (i32, [vp, u64, u32, C.POINTER(vp)]),
            "skq_session_free": (i32, [vp]),
            "skq_sketch": (i32, [vp, vp, vp, u32, u64, u32, u32, vp]),
            "skq_sketch_seqs": (i32, [vp, vp, vp, u32, u64, u32, u32, vp]),
            "skq_sketcher_create": (i32, [i32, u64, C.POINTER(vp)]),
            "skq_sketcher_run": (i32, [vp, C.c_char_p, u64, u32, u32, vp, u64, C.POINTER(u64)]),
            "skq_sketcher_free": (i32, [vp]),
            "skq_chain": (i32, [vp, dbl, i32, vp]),
            "skq_map": (i32, [vp, vp, vp, u32, u64, u32, u32, dbl, i32, vp]),
            "skq_chain_sketches": (i32, [vp, u64, vp, vp, vp, vp, dbl, i32, vp]),
            "skq_session_results": (i32, [vp, C.POINTER(_Results)]),
            "skq_session_check": (i32, [vp, vp]),
            "skq_session_reset_totals": (i32, [vp, vp]),
            "skq_session_export": (i32, [vp] + [vp] * 6 + [C.POINTER(u64), C.POINTER(u64)]),
            "skq_session_totals": (i32, [vp, vp, vp, i32, vp]),
            "skq_session_totals_async": (i32, [vp, vp, vp, vp]),
            "skq_malloc": (i32, [i32, C.c_size_t, C.POINTER(vp)]),
            "skq_free": (i32, [vp]),
            "skq_memcpy_h2d": (i32, [vp, vp, C.c_size_t, vp]),
            "skq_memcpy_d2h": (i32, [vp, vp, C.c_size_t, vp]),
            "skq_stream_sync": (i32, [vp]),
            "skq_session_enable_timing": (i32, [vp, i32]),
            "skq_session_set_stamps": (i32, [vp, vp]),
            "skq_session_kernel_time": (i32, [vp, i32, C.POINTER(dbl), C.POINTER(u64)]),
            "skq_tables_build": (i32, [u32, vp, vp, u32, vp, u32, i32, C.POINTER(vp)]),
            "skq_tables_build_gpu": (i32, [i32, u32, vp, vp, u32, vp, u32, C.POINTER(vp)]),
            "skq_tables_count": (u32, [vp]),
            "skq_tables_get": (i32, [vp, u32, C.POINTER(_KmerTable)]),
            "skq_tables_free": (i32, [vp]),
            "skq_host_sketch": (C.c_int64, [vp, u64, u32, u32, vp]),
            "skq_fasta_load": (i32, [C.c_char_p, C.POINTER(vp)]),
            "skq_seqs_count": (u64, [vp]),
            "skq_seqs_view": (i32, [vp] + [C.POINTER(vp)] * 4),
            "skq_seqs_free": (i32, [vp]),
            "skq_fastq_open": (i32, [C.c_char_p, C.POINTER(vp)]),
            "skq_fastq_next": (i32, [vp, u64, C.POINTER(u64), C.POINTER(vp), C.POINTER(vp), C.POINTER(u64)]),
            "skq_fastq_mark": (i32, [vp, u64, u64, vp]),
            "skq_fastq_kept": (i32, [vp, u64]),
            "skq_fastq_records": (u64, [vp]),
            "skq_fastq_id": (i32, [vp, u64, C.POINTER(vp), C.POINTER(u64)]),
            "skq_fastq_close": (i32, [vp]),
            "skq_ingest_open": (i32, [vp, C.c_char_p, u64, i32, C.POINTER(vp)]),
            "skq_ingest_open_range": (i32, [vp, C.c_char_p, u64, u64, C.c_uint32, u64, i32, C.POINTER(vp)]),
            "skq_ingest_supersede": (i32, [vp, C.c_uint32, vp]),
            "skq_fastq_split": (i32, [C.c_char_p, C.c_uint32, vp, vp]),
            "skq_ingest_map": (i32, [vp, u32, dbl, i32, vp, C.POINTER(u64), C.POINTER(u64)]),
            "skq_ingest_records": (u64, [vp]),
            "skq_ingest_finish": (i32, [vp, vp]),
            "skq_ingest_id": (i32, [vp, u64, C.POINTER(vp), C.POINTER(u64)]),
            "skq_ingest_close": (i32, [vp]),
            "skq_legacy_index_write": (i32, [C.c_char_p, u32, vp, vp, vp]),
            "skq_legacy_index_read": (i32, [C.c_char_p, C.POINTER(vp)]),
            "skq_legacy_index_view": (i32, [vp, C.POINTER(u32), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]),
            "skq_legacy_index_free": (i32, [vp]),
            "skq_sidecar_write": (i32, [C.c_char_p, u32, vp, vp, vp]),
            "skq_index_open": (i32, [C.c_char_p, C.POINTER(vp), C.POINTER(i32)]),
            "skq_em": (i32, [u64, vp, vp, vp, u32, i32, dbl, i32, vp, C.POINTER(i32)]),
            "skq_assign": (i32, [u64, vp, vp, vp, u32, vp, vp, vp]),
            "skq_csv_write": (i32, [C.c_char_p, vp, vp, vp, vp]),
            "skq_em_create": (i32, [i32, u32, C.POINTER(vp)]),
            "skq_em_free": (i32, [vp]),
            "skq_em_add": (i32, [vp, u64, vp, vp, vp]),
            "skq_em_add_session": (i32, [vp, vp, vp]),
            "skq_em_size": (u64, [vp]),
            "skq_em_select": (i32, [vp, vp]),
            "skq_em_reads": (u64, [vp]),
            "skq_em_init": (i32, [vp, vp, vp]),
            "skq_em_estep": (i32, [vp, vp, vp, vp]),
            "skq_em_mstep": (i32, [vp, vp, vp, u64, C.POINTER(dbl), vp]),
            "skq_em_run": (i32, [vp, i32, dbl, vp, C.POINTER(i32)]),
            "skq_em_assign": (i32, [vp, vp, vp, vp, vp]),
            "skq_em_assign_host": (i32, [vp, vp, vp, vp]),
            "skq_em_estep_host": (i32, [u64, vp, vp, vp, u32, vp, i32, vp]),
            "skq_em_mstep_host": (i32, [u32, vp, vp, u64, C.POINTER(dbl)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise SkqError("skq error %d: %s" % (rc, lib().skq_last_error().decode()))


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def threshold(fraction=float(np.float32(0.05))):
    """(uint32_t)(UINT32_MAX * fraction); quant passes (double)0.05f (src/main.cpp:43)."""
    return lib().skq_threshold(fraction)


class DeviceBuffer:
    """Raw device allocation through the C ABI (no torch needed)."""

    def __init__(self, nbytes, device=0):
        self.nbytes = int(nbytes)
        self.ptr = C.c_void_p()
        _check(lib().skq_malloc(device, max(self.nbytes, 1), C.byref(self.ptr)))

    @classmethod
    def from_numpy(cls, a, device=0):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, device)
        if a.nbytes:
            _check(lib().skq_memcpy_h2d(b.ptr, _p(a), a.nbytes, None))
            _check(lib().skq_stream_sync(None))
        return b

    def to_numpy(self, dtype, count):
        out = np.empty(count, dtype)
        if out.nbytes:
            _check(lib().skq_memcpy_d2h(_p(out), self.ptr, out.nbytes, None))
        return out

    @property
    def value(self):
        return self.ptr.value

    def free(self):
        if self.ptr:
            lib().skq_free(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Index:
    """Device-resident inverted index. tables: {k: (keys u32 asc, offs u64 [nkeys+1], tids u32)}."""

    def __init__(self, ks, ntx, tables, device=0, seqs=None, thr=None):
        """seqs = (flat bytes, offs[ntx + 1]): the transcripts the tables were built from; they add
        the chained tables, one per k slot (skq_index_create_chained; SKQ_CHAIN), sketched at thr."""
        self.ks = [int(k) for k in ks]
        self.ntx = int(ntx)
        self.device = device
        self._keep = []
        arr = (_KmerTable * len(tables))()
        for j, (k, (keys, offs, tids)) in enumerate(tables.items()):
            keys = np.ascontiguousarray(keys, np.uint32)
            offs = np.ascontiguousarray(offs, np.uint64)
            tids = np.ascontiguousarray(tids, np.uint32)
            self._keep += [keys, offs, tids]
            arr[j] = _KmerTable(int(k), len(keys), _p(keys), _p(offs), _p(tids))
        ka = np.array(self.ks, np.uint32)
        self.h = C.c_void_p()
        if seqs is None:
            _check(lib().skq_index_create(device, self.ntx, len(self.ks), _p(ka), len(tables),
                                          C.cast(arr, C.c_void_p), C.byref(self.h)))
        else:
            sb = np.ascontiguousarray(seqs[0], np.uint8)
            so = np.ascontiguousarray(seqs[1], np.uint64)
            _check(lib().skq_index_create_chained(device, self.ntx, len(self.ks), _p(ka), len(tables),
                                                  C.cast(arr, C.c_void_p), _p(sb), _p(so), len(so) - 1,
                                                  threshold() if thr is None else thr, C.byref(self.h)))
        self._keep = None

    def stats(self):
        b, n, m = C.c_uint64(), C.c_uint64(), C.c_uint32()
        _check(lib().skq_index_stats(self.h, C.byref(b), C.byref(n), C.byref(m)))
        cs, cb = C.c_double(), C.c_uint64()
        _check(lib().skq_index_chain_build(self.h, C.byref(cs), C.byref(cb)))
        return dict(device_bytes=b.value, postings=n.value, max_list=m.value,
                    direct=bool(lib().skq_index_direct(self.h)),
                    probe={0: "bucket", 1: "dir", 2: "rank", 3: "wide", 5: "compact"}[lib().skq_index_direct(self.h)],
                    chained=lib().skq_index_chained(self.h), chain_build_s=round(cs.value, 3),
                    chain_host_peak_bytes=cb.value)

    def free(self):
        if self.h:
            lib().skq_index_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Session:
    def __init__(self, index, max_reads, max_len):
        self.index = index
        self.h = C.c_void_p()
        _check(lib().skq_session_create(index.h, int(max_reads), int(max_len), C.byref(self.h)))

    def sketch(self, d_reads, d_offs, n_reads, max_len, fixed_len=0, thr=None, stream=None,
               nthash=False):
        """nthash=False: quant reads (invalid/short reads rejected); True: createSketch on any
        sequence (invalid-base windows skipped)."""
        thr = threshold() if thr is None else thr
        f = lib().skq_sketch_seqs if nthash else lib().skq_sketch
        _check(f(self.h, d_reads, d_offs, fixed_len, n_reads, max_len, thr, stream))

    def chain(self, fraction=0.9, accumulate=True, stream=None):
        _check(lib().skq_chain(self.h, fraction, int(accumulate), stream))

    def map(self, d_reads, d_offs, n_reads, max_len, fixed_len=0, thr=None, fraction=0.9,
            accumulate=True, stream=None):
        thr = threshold() if thr is None else thr
        _check(lib().skq_map(self.h, d_reads, d_offs, fixed_len, n_reads, max_len, thr, fraction,
                             int(accumulate), stream))

    def chain_sketches(self, n_reads, d_hashes, d_offs, d_cnt, d_present=None, fraction=0.9,
                       accumulate=True, stream=None):
        _check(lib().skq_chain_sketches(self.h, n_reads, d_hashes, d_offs, d_cnt, d_present, fraction,
                                        int(accumulate), stream))

    def check(self, stream=None):
        _check(lib().skq_session_check(self.h, stream))

    def results(self):
        r = _Results()
        _check(lib().skq_session_results(self.h, C.byref(r)))
        return r

    def export(self):
        nh, nc = C.c_uint64(), C.c_uint64()
        _check(lib().skq_session_export(self.h, None, None, None, None, None, None, C.byref(nh), C.byref(nc)))
        r = self.results()
        n, nk = r.n_reads, r.nk
        st = np.zeros(max(n, 1), np.uint8)
        ho = np.zeros(n * nk + 1, np.uint64)
        hs = np.zeros(max(nh.value, 1), np.uint32)
        co = np.zeros(n + 1, np.uint64)
        ct = np.zeros(max(nc.value, 1), np.uint32)
        cs = np.zeros(max(nc.value, 1), np.uint32)
        _check(lib().skq_session_export(self.h, _p(st), _p(ho), _p(hs), _p(co), _p(ct), _p(cs),
                                        C.byref(nh), C.byref(nc)))
        return dict(status=st[:n], hash_offs=ho, hashes=hs[:nh.value], cand_offs=co,
                    cand_tid=ct[:nc.value], cand_score=cs[:nc.value], nk=nk)

    def totals(self):
        ntx = self.index.ntx
        a = np.zeros(max(ntx, 1), np.uint64)
        b = np.zeros(max(ntx, 1), np.uint64)
        _check(lib().skq_session_totals(self.h, _p(a), _p(b), 0, None))
        return a[:ntx], b[:ntx]

    def totals_to_device(self, d_reads_ptr, d_score_ptr, stream=None):
        _check(lib().skq_session_totals(self.h, d_reads_ptr, d_score_ptr, 1, stream))

    def totals_async(self, d_reads_ptr, d_score_ptr, stream=None):
        """The totals into device memory on the session's tail stream, after `stream`'s work so far,
        with `stream` waiting for the copy (include/skq.h skq_session_totals_async): the next map
        does not wait for it."""
        _check(lib().skq_session_totals_async(self.h, d_reads_ptr, d_score_ptr, stream))

    def reset_totals(self, stream=None):
        _check(lib().skq_session_reset_totals(self.h, stream))

    def set_stamps(self, d_ptr):
        """Development: k_map1 phase clocks into a device buffer of 8 u64 per wave (0 = off)."""
        _check(lib().skq_session_set_stamps(self.h, d_ptr or None))

    def enable_timing(self, on=True):
        _check(lib().skq_session_enable_timing(self.h, int(on)))

    def slow_reads(self):
        """(sketch slow-path reads, chain slow-path reads) of the last batch."""
        a, b = C.c_uint32(), C.c_uint32()
        _check(lib().skq_session_slow_reads(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def slow_counts(self):
        """(sketch slow, chain slow, second-level sketch, second-level chain) reads of the last batch."""
        c = (C.c_uint32 * 4)()
        _check(lib().skq_session_slow_counts(self.h, c))
        return tuple(c)

    def kernel_time(self, kind):
        ms, n = C.c_double(), C.c_uint64()
        _check(lib().skq_session_kernel_time(self.h, kind, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def free(self):
        if self.h:
            lib().skq_session_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def build_tables(seqs, offs, ks, thr=None, nthreads=0):
    """Host index builder (product C++): sketch transcripts seqs[offs[t]:offs[t+1]] at every
    k and invert. Returns {k: (keys, offs, tids)} as numpy arrays."""
    thr = threshold() if thr is None else thr
    seqs = np.ascontiguousarray(seqs, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    ka = np.array(ks, np.uint32)
    h = C.c_void_p()
    _check(lib().skq_tables_build(len(offs) - 1, _p(seqs), _p(offs), len(ka), _p(ka), thr, nthreads,
                                  C.byref(h)))
    try:
        return _tables_dict(h)
    finally:
        lib().skq_tables_free(h)


def build_tables_gpu(seqs, offs, ks, thr=None, device=0):
    """The same tables as build_tables, built on the GPU (skq_tables_build_gpu)."""
    thr = threshold() if thr is None else thr
    seqs = np.ascontiguousarray(seqs, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    ka = np.array(ks, np.uint32)
    h = C.c_void_p()
    _check(lib().skq_tables_build_gpu(device, len(offs) - 1, _p(seqs), _p(offs), len(ka), _p(ka), thr, C.byref(h)))
    try:
        return _tables_dict(h)
    finally:
        lib().skq_tables_free(h)


def _arr(ptr, ctype, count, dtype):
    if count == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), (count,)).astype(dtype, copy=True)


def _tables_dict(h):
    out = {}
    for i in range(lib().skq_tables_count(h)):
        t = _KmerTable()
        _check(lib().skq_tables_get(h, i, C.byref(t)))
        n = t.nkeys
        offs_a = _arr(t.offs, C.c_uint64, n + 1, np.uint64)
        out[int(t.k)] = (_arr(t.keys, C.c_uint32, n, np.uint32), offs_a,
                         _arr(t.tids, C.c_uint32, int(offs_a[-1]), np.uint32))
    return out


def _seqs(h):
    """(names, sequences) of a skq_seqs handle, as lists of bytes."""
    n = lib().skq_seqs_count(h)
    sb, so, nb, no = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
    _check(lib().skq_seqs_view(h, C.byref(sb), C.byref(so), C.byref(nb), C.byref(no)))
    so_a = _arr(so, C.c_uint64, n + 1, np.uint64)
    no_a = _arr(no, C.c_uint64, n + 1, np.uint64)
    seq_b = C.string_at(sb, int(so_a[-1])) if so_a[-1] else b""
    name_b = C.string_at(nb, int(no_a[-1])) if no_a[-1] else b""
    return ([name_b[no_a[i]:no_a[i + 1]] for i in range(n)], [seq_b[so_a[i]:so_a[i + 1]] for i in range(n)])


def fasta_load(path):
    """load_fasta (src/data_io.cpp:47-80): (names, sequences) in file order."""
    h = C.c_void_p()
    _check(lib().skq_fasta_load(str(path).encode(), C.byref(h)))
    try:
        return _seqs(h)
    finally:
        lib().skq_seqs_free(h)


def csv_write(path, fasta_path, counts, assigned, pi):
    """output_to_csv (src/data_io.cpp:133-152) through skq_csv_write, for the transcripts of
    fasta_path (load_fasta order = dense ids)."""
    h = C.c_void_p()
    _check(lib().skq_fasta_load(str(fasta_path).encode(), C.byref(h)))
    try:
        c = np.ascontiguousarray(counts, np.float64)
        a = np.ascontiguousarray(assigned, np.uint8)
        p = np.ascontiguousarray(pi, np.float64)
        _check(lib().skq_csv_write(str(path).encode(), h, _p(c), _p(a), _p(p)))
    finally:
        lib().skq_seqs_free(h)


def legacy_index_read(path):
    """load_index (src/data_io.cpp:233-304): (ks, names, sequences, {k: (keys, offs, tids)})."""
    h = C.c_void_p()
    _check(lib().skq_legacy_index_read(str(path).encode(), C.byref(h)))
    try:
        nk, ks, tx, tabs = C.c_uint32(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        _check(lib().skq_legacy_index_view(h, C.byref(nk), C.byref(ks), C.byref(tx), C.byref(tabs)))
        names, seqs = _seqs(tx)
        return ([int(x) for x in _arr(ks, C.c_uint32, nk.value, np.uint32)], names, seqs, _tables_dict(tabs))
    finally:
        lib().skq_legacy_index_free(h)


def index_open(path):
    """quant's index loader (skq_index_open): the `<path>.skq` sidecar when its stamp matches the
    legacy file, else the legacy file. (ks, names, sequences, tables, from_sidecar); sequences
    are empty when read from the sidecar."""
    h = C.c_void_p()
    side = C.c_int()
    _check(lib().skq_index_open(str(path).encode(), C.byref(h), C.byref(side)))
    try:
        nk, ks, tx, tabs = C.c_uint32(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        _check(lib().skq_legacy_index_view(h, C.byref(nk), C.byref(ks), C.byref(tx), C.byref(tabs)))
        names, seqs = _seqs(tx)
        return ([int(x) for x in _arr(ks, C.c_uint32, nk.value, np.uint32)], names, seqs, _tables_dict(tabs),
                bool(side.value))
    finally:
        lib().skq_legacy_index_free(h)


class FastqReader:
    """process_fastq_single_pass's record reader (src/main.cpp:113-148), in batches."""

    def __init__(self, path):
        self.h = C.c_void_p()
        _check(lib().skq_fastq_open(str(path).encode(), C.byref(self.h)))

    def next(self, max_reads):
        """(first ordinal, [sequence bytes]) of the next batch ([] at the end)."""
        n, b, o, first = C.c_uint64(), C.c_void_p(), C.c_void_p(), C.c_uint64()
        _check(lib().skq_fastq_next(self.h, max_reads, C.byref(n), C.byref(b), C.byref(o), C.byref(first)))
        offs = _arr(o, C.c_uint64, n.value + 1, np.uint64) if n.value else np.zeros(1, np.uint64)
        data = C.string_at(b, int(offs[-1])) if offs[-1] else b""
        return first.value, [data[offs[i]:offs[i + 1]] for i in range(n.value)]

    def mark(self, first, status):
        st = np.ascontiguousarray(status, np.uint8)
        _check(lib().skq_fastq_mark(self.h, first, len(st), _p(st)))

    def kept(self, ordinal):
        return bool(lib().skq_fastq_kept(self.h, ordinal))

    def id(self, ordinal):
        p, n = C.c_void_p(), C.c_uint64()
        _check(lib().skq_fastq_id(self.h, ordinal, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value)

    def close(self):
        if self.h:
            lib().skq_fastq_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()


class Ingest:
    """FASTQ parsed on the GPU (skq_ingest_*): batches of records mapped through `session`."""

    def __init__(self, session, path, chunk_bytes=0, io_threads=0, part=None):
        """part = (lo, hi, entry_state): only the records whose header starts in [lo, hi)
        (fastq_split), numbered from 0."""
        self.session = session  # keeps the session alive
        self.h = C.c_void_p()
        if part is None:
            _check(lib().skq_ingest_open(session.h, str(path).encode(), chunk_bytes, io_threads, C.byref(self.h)))
        else:
            lo, hi, state = part
            _check(lib().skq_ingest_open_range(session.h, str(path).encode(), lo, hi, state, chunk_bytes, io_threads,
                                               C.byref(self.h)))

    def map(self, thr=None, fraction=0.9, accumulate=True, stream=None):
        """(first ordinal, n) of the next batch, now in the session's results; n == 0 at the end."""
        n, first = C.c_uint64(), C.c_uint64()
        _check(lib().skq_ingest_map(self.h, threshold() if thr is None else thr, fraction, int(accumulate),
                                    stream, C.byref(n), C.byref(first)))
        return first.value, n.value

    def records(self):
        return lib().skq_ingest_records(self.h)

    def finish(self):
        kept = np.zeros(self.records(), np.uint8)
        _check(lib().skq_ingest_finish(self.h, _p(kept)))
        return kept

    def id(self, ordinal):
        p, n = C.c_void_p(), C.c_uint64()
        _check(lib().skq_ingest_id(self.h, ordinal, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value)

    def close(self):
        if self.h:
            lib().skq_ingest_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()


def fastq_split(path, parts):
    """(offs[parts + 1], states[parts]): the file's parts at line starts with the reader's exact
    state at each (skq_fastq_split)."""
    offs = np.zeros(parts + 1, np.uint64)
    states = np.zeros(parts, np.uint32)
    _check(lib().skq_fastq_split(str(path).encode(), parts, _p(offs), _p(states)))
    return offs, states


def ingest_supersede(ingests, kepts):
    """Clear kept flags of records whose id a later part keeps (skq_ingest_supersede)."""
    hs = (C.c_void_p * len(ingests))(*[g.h.value for g in ingests])
    ks = (C.c_void_p * len(kepts))(*[k.ctypes.data for k in kepts])
    _check(lib().skq_ingest_supersede(C.cast(hs, C.c_void_p), len(ingests), C.cast(ks, C.c_void_p)))


def _csr(cand_offs, cand_tid, cand_score):
    return (np.ascontiguousarray(cand_offs, np.uint64), np.ascontiguousarray(cand_tid, np.uint32),
            np.ascontiguousarray(cand_score, np.uint32))


class EMSet:
    """One device's share of the reads' candidate lists for the GPU EM (skq_em_*; include/skq.h).

    add(offs, tid, score) / add_session(session) append reads in order; select(keep) keeps a
    subset; run() and assign() do the whole thing on one device. estep / mstep take device
    pointers (e.g. torch tensors' data_ptr()) for the multi-GPU loop in skq/dist.py."""

    def __init__(self, ntx, device=0):
        self.ntx = int(ntx)
        self.device = device
        self.h = C.c_void_p()
        _check(lib().skq_em_create(device, self.ntx, C.byref(self.h)))

    def add(self, cand_offs, cand_tid, cand_score):
        o, t, s = _csr(cand_offs, cand_tid, cand_score)
        _check(lib().skq_em_add(self.h, len(o) - 1, _p(o), _p(t), _p(s)))

    def add_session(self, session, stream=None):
        _check(lib().skq_em_add_session(self.h, session.h, stream))

    def size(self):
        return lib().skq_em_size(self.h)

    def select(self, keep):
        k = np.ascontiguousarray(keep, np.uint8)
        _check(lib().skq_em_select(self.h, _p(k)))

    def reads(self):
        return lib().skq_em_reads(self.h)

    def init(self, d_pi, stream=None):
        _check(lib().skq_em_init(self.h, d_pi, stream))

    def estep(self, d_pi, d_post, stream=None):
        _check(lib().skq_em_estep(self.h, d_pi, d_post, stream))

    def mstep(self, d_pi, d_post, total_reads, stream=None):
        ch = C.c_double()
        _check(lib().skq_em_mstep(self.h, d_pi, d_post, int(total_reads), C.byref(ch), stream))
        return ch.value

    def run(self, max_iterations=20, convergence=0.01):
        """(pi, iterations) on this device alone."""
        pi = np.zeros(self.ntx, np.float64)
        it = C.c_int()
        _check(lib().skq_em_run(self.h, max_iterations, convergence, _p(pi), C.byref(it)))
        return pi, it.value

    def assign_device(self, d_pi, d_counts, d_assigned, stream=None):
        _check(lib().skq_em_assign(self.h, d_pi, d_counts, d_assigned, stream))

    def assign(self, pi=None):
        """(counts, assigned) for pi (host; None = the pi run() left on the device)."""
        counts = np.zeros(self.ntx, np.float64)
        assigned = np.zeros(self.ntx, np.uint8)
        p = None if pi is None else np.ascontiguousarray(pi, np.float64)
        _check(lib().skq_em_assign_host(self.h, _p(p), _p(counts), _p(assigned)))
        return counts, assigned.astype(bool)

    def free(self):
        if self.h:
            lib().skq_em_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def em_estep_host(cand_offs, cand_tid, cand_score, ntx, pi):
    """Posterior sums of these reads under pi (host E-step; the CPU side of skq/dist.py's EM)."""
    o, t, s = _csr(cand_offs, cand_tid, cand_score)
    pi = np.ascontiguousarray(pi, np.float64)
    post = np.zeros(max(ntx, 1), np.float64)
    _check(lib().skq_em_estep_host(len(o) - 1, _p(o), _p(t), _p(s), ntx, _p(pi), 1, _p(post)))
    return post[:ntx]


def em_mstep_host(pi, post, total_reads):
    """M-step in place on pi (float64, contiguous); returns the change."""
    assert pi.dtype == np.float64 and pi.flags.c_contiguous
    post = np.ascontiguousarray(post, np.float64)
    ch = C.c_double()
    _check(lib().skq_em_mstep_host(len(pi), _p(pi), _p(post), int(total_reads), C.byref(ch)))
    return ch.value


def em(cand_offs, cand_tid, cand_score, ntx, max_iterations=20, convergence=0.01, nthreads=0):
    """estimate_isoform_abundance_em (src/isoform_assignment.cpp:9-65): (pi, iterations)."""
    o, t, s = _csr(cand_offs, cand_tid, cand_score)
    pi = np.zeros(max(ntx, 1), np.float64)
    it = C.c_int()
    _check(lib().skq_em(len(o) - 1, _p(o), _p(t), _p(s), ntx, max_iterations, convergence, nthreads, _p(pi),
                        C.byref(it)))
    return pi[:ntx], it.value


def assign(cand_offs, cand_tid, cand_score, ntx, pi):
    """assign_reads_to_isoforms (src/isoform_assignment.cpp:67-97): (counts, assigned)."""
    o, t, s = _csr(cand_offs, cand_tid, cand_score)
    pi = np.ascontiguousarray(pi, np.float64)
    counts = np.zeros(max(ntx, 1), np.float64)
    assigned = np.zeros(max(ntx, 1), np.uint8)
    _check(lib().skq_assign(len(o) - 1, _p(o), _p(t), _p(s), ntx, _p(pi), _p(counts), _p(assigned)))
    return counts[:ntx], assigned[:ntx].astype(bool)


class Sketcher:
    """One sequence per call (skq_sketcher_run): the per-sequence path the C++ drop-in serves."""

    def __init__(self, device=0, max_len=4096):
        self.h = C.c_void_p()
        _check(lib().skq_sketcher_create(device, max_len, C.byref(self.h)))

    def run(self, seq: bytes, k: int, thr=None):
        """The retained windows' hashes (unordered, repeats kept) as uint32."""
        t = threshold() if thr is None else thr
        nw = max(0, len(seq) - k + 1) if k > 0 else 0
        out = np.empty(max(nw, 1), np.uint32)
        n = C.c_uint64()
        _check(lib().skq_sketcher_run(self.h, seq, len(seq), k, t, _p(out), nw, C.byref(n)))
        return out[:min(n.value, nw)]

    def free(self):
        if self.h:
            lib().skq_sketcher_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def host_sketch(seq: bytes, k: int, thr=None):
    thr = threshold() if thr is None else thr
    a = np.frombuffer(seq, np.uint8) if seq else np.zeros(1, np.uint8)
    out = np.zeros(max(len(seq), 1), np.uint32)
    m = lib().skq_host_sketch(_p(a), len(seq), k, thr, _p(out))
    if m < 0:
        raise SkqError("len < k or k == 0")
    return [int(x) for x in out[:m]]


def pack_reads(reads):
    """list of bytes -> (uint8 buffer, uint64 offsets)"""
    buf = np.frombuffer(b"".join(reads) or b"\0", np.uint8).copy()
    offs = np.zeros(len(reads) + 1, np.uint64)
    if reads:
        offs[1:] = np.cumsum([len(r) for r in reads])
    return buf, offs
