"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact.

Every comparison is exact: retained-hash sets per (read, k), per-read status, and candidate
lists (tid, score) in the normalised order (score desc, tid asc).
"""
import ctypes as C
import random
import sys

import numpy as np
import pytest

import orc
import skq
from skq import synth

pytestmark = pytest.mark.gpu
SPLIT = False  # run_gpu: sketch and chain as two calls instead of skq_map (the wide-split mode)
CHAINED = False  # build: indexes from sequences get the chained tables (skq_index_create_chained)


@pytest.fixture(autouse=True, params=["chain", "chain-compact", "compact", "compact-split",
                                      "wide", "wide-split", "dir", "rank", "bucket"])
def probe_mode(request, monkeypatch):
    """Every test runs with each index probe structure: compact (minimal-perfect-hash) tables
    and wide direct tables gathered by the map or count kernel, 4-B direct and rank tables
    (transcript ids past 2^22) probed inside the sketch kernel, and the bucket table probed by k_probe
    (SKQ_DIRECT_MB=0). "-split": the same tables through skq_sketch + skq_chain (no fused map).
    "chain": wide tables plus the chained tables (SKQ_CHAIN=1, one per k slot of indexes built
    from sequences, up to 4 slots); other indexes run as wide. "chain-compact": the chained
    tables over compact tables (entries at the keys' compact slots, k_map1 TAB 4)."""
    if request.param.startswith("chain"):
        # chained tables (per k slot, indexes built from sequences) over wide or compact tables
        monkeypatch.setenv("SKQ_DIRECT_MB", "49152")
        monkeypatch.setenv("SKQ_PROBE", "compact" if request.param == "chain-compact" else "wide")
        monkeypatch.setenv("SKQ_CHAIN", "1")
        monkeypatch.setattr(sys.modules[__name__], "CHAINED", True)
    elif request.param == "bucket":
        monkeypatch.setenv("SKQ_DIRECT_MB", "0")
    elif request.param.endswith("-split"):
        monkeypatch.setenv("SKQ_DIRECT_MB", "49152")
        monkeypatch.setenv("SKQ_PROBE", request.param.split("-")[0])
        monkeypatch.setattr(sys.modules[__name__], "SPLIT", True)
    else:
        monkeypatch.setenv("SKQ_DIRECT_MB", "49152")
        monkeypatch.setenv("SKQ_PROBE", request.param)
    return request.param


def build(ks, seqs=None, tx=None, pairs=None, ntx=None):
    """(product device index, oracle index) over the same transcripts / postings."""
    if pairs is not None:
        tables = {}
        for k, (h, t) in zip(ks, pairs):
            order = np.lexsort((t, h))
            h, t = np.asarray(h, np.uint32)[order], np.asarray(t, np.uint32)[order]
            keep = np.ones(len(h), bool)
            keep[1:] = (h[1:] != h[:-1]) | (t[1:] != t[:-1])
            h, t = h[keep], t[keep]
            keys, first = np.unique(h, return_index=True)
            offs = np.append(first, len(h)).astype(np.uint64)
            tables[k] = (keys, offs, t)
        return skq.Index(ks, ntx, tables), orc.Index(ks, pairs=pairs, ntx=ntx)
    if tx is not None:
        seqs = [tx.seq(t) for t in range(tx.ntx)]
    buf, offs = skq.pack_reads(seqs)
    tables = skq.build_tables(buf, offs, ks)
    return (skq.Index(ks, len(seqs), tables, seqs=(buf, offs) if CHAINED else None),
            orc.Index(ks, seqs=seqs))


def run_gpu(index, reads, fixed_len=0, fraction=0.9, thr=None, max_len=None):
    buf, offs = skq.pack_reads(reads)
    n = len(reads)
    max_len = max_len if max_len is not None else max([len(r) for r in reads] + [1])
    s = skq.Session(index, max(n, 1), max_len)
    d_buf = skq.DeviceBuffer.from_numpy(buf)
    d_offs = None if fixed_len else skq.DeviceBuffer.from_numpy(offs)
    if SPLIT:
        s.sketch(d_buf.ptr, d_offs.ptr if d_offs else None, n, max_len, fixed_len=fixed_len, thr=thr)
        s.chain(fraction=fraction)
    else:
        s.map(d_buf.ptr, d_offs.ptr if d_offs else None, n, max_len, fixed_len=fixed_len, thr=thr,
              fraction=fraction)
    s.check()
    out = s.export()
    out["totals"] = s.totals()
    return out


def compare(out, ref, n, nk, check_hashes=True):
    np.testing.assert_array_equal(out["status"], ref["status"][:n])
    ho = out["hash_offs"]
    co = out["cand_offs"]
    for r in range(n):
        if check_hashes:
            for i in range(nk):
                e = r * nk + i
                got = out["hashes"][ho[e]:ho[e + 1]]
                exp = ref["hashes"][r, i, :ref["hash_cnt"][r, i]]
                assert list(got) == list(exp), (r, i)
        gt = out["cand_tid"][co[r]:co[r + 1]]
        gs = out["cand_score"][co[r]:co[r + 1]]
        c = ref["cand_cnt"][r]
        assert list(gt) == list(ref["cand_tid"][r, :c]), r
        assert list(gs) == list(ref["cand_score"][r, :c]), r


def totals_from(ref, n, ntx):
    tr = np.zeros(ntx, np.uint64)
    ts = np.zeros(ntx, np.uint64)
    for r in range(n):
        c = ref["cand_cnt"][r]
        for j in range(c):
            tr[ref["cand_tid"][r, j]] += 1
            ts[ref["cand_tid"][r, j]] += ref["cand_score"][r, j]
    return tr, ts


def test_probe_mode_is_selected(tx300, probe_mode):
    gi, _ = build([21, 31], tx=tx300)
    st = gi.stats()
    base = {"chain": "wide", "chain-compact": "compact"}.get(probe_mode, probe_mode.split("-")[0])
    assert st["probe"] == base
    assert st["device_bytes"] > 0
    assert (st["chained"] > 1) == probe_mode.startswith("chain")  # (one chained table per k slot)
    gi1, _ = build([31], tx=tx300)
    assert (gi1.stats()["chained"] > 1) == probe_mode.startswith("chain")


@pytest.fixture(scope="module")
def tx300():
    return synth.transcriptome(300, seed=21)


@pytest.mark.parametrize("ks", [[31], [21, 25, 31], [31, 31], [19], [17, 19, 21, 25, 31]])
@pytest.mark.parametrize("read_len", [100, 150, 250])
def test_random_reads_match_oracle(tx300, ks, read_len):
    gi, oi = build(ks, tx=tx300)
    bases, _, _ = synth.reads(tx300, 3000, read_len, seed=read_len + len(ks), err=0.002)
    reads = [bases[i * read_len:(i + 1) * read_len].tobytes() for i in range(3000)]
    out = run_gpu(gi, reads)
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), len(ks))
    tr, ts = totals_from(ref, len(reads), tx300.ntx)
    np.testing.assert_array_equal(out["totals"][0], tr)
    np.testing.assert_array_equal(out["totals"][1], ts)
    assert (ref["cand_cnt"] > 0).mean() > 0.9


def test_fixed_length_mode_equals_offsets_mode(tx300):
    gi, oi = build([31], tx=tx300)
    bases, _, _ = synth.reads(tx300, 2049, 150, seed=5)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(2049)]
    a = run_gpu(gi, reads, fixed_len=150)
    ref = oi.map_batch(reads)
    compare(a, ref, len(reads), 1)


def test_edge_reads(tx300):
    gi, oi = build([31], tx=tx300)
    base = tx300.seq(3)
    rng = random.Random(1)
    reads = [
        b"",                                   # empty: valid but short
        base[:30],                             # short
        base[:31],                             # exactly k
        base[:150].lower(),                    # lowercase: invalid
        base[:70] + b"N" + base[71:150],       # N: invalid
        base[:149] + b"\r",                    # trailing CR: invalid
        base[:150] + b" ",                     # trailing space: invalid
        base[:300],                            # > 256: slow path
        base[:257],
        base[:256],
        b"A" * 150,                            # low complexity
        (b"ACGT" * 70)[:280],
        bytes(rng.choice(b"ACGT") for _ in range(150)),
        base[10:160],
    ]
    reads += [base[j:j + 40] for j in range(0, 200, 7)]
    out = run_gpu(gi, reads)
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), 1)


def test_variable_lengths_and_unaligned(tx300):
    gi, oi = build([21, 31], tx=tx300)
    rng = random.Random(7)
    reads = []
    for _ in range(1500):
        t = rng.randrange(tx300.ntx)
        s = tx300.seq(t)
        L = rng.randint(0, min(len(s), 400))
        p = rng.randint(0, len(s) - L)
        reads.append(s[p:p + L])
    out = run_gpu(gi, reads)
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), 2)


def test_many_retained_hashes_take_slow_path():
    # a high sketch fraction forces more than HCAP retained hashes per read
    tx = synth.transcriptome(80, seed=3)
    thr = orc.threshold(0.5)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    buf, offs = skq.pack_reads(seqs)
    gi = skq.Index([31], len(seqs), skq.build_tables(buf, offs, [31], thr=thr))
    oi = orc.Index([31], seqs=seqs, thr=thr)
    bases, _, _ = synth.reads(tx, 500, 150, seed=4)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(500)]
    out = run_gpu(gi, reads, thr=thr)
    ref = oi.map_batch(reads, thr=thr)
    compare(out, ref, len(reads), 1)


def test_sketch_seqs_follows_nthash_semantics(tx300):
    """skq_sketch_seqs = createSketch_FracMinhash_direct on arbitrary sequences: windows with a
    byte outside ACGTUacgtu skipped, lowercase and U hashed like uppercase / T, nothing rejected."""
    ks = [21, 25, 31]
    gi, _ = build(ks, tx=tx300)
    rng = random.Random(17)
    alpha = b"ACGTACGTACGTacgtUuN\x01\x03R\r"
    seqs = [tx300.seq(3)[:400], tx300.seq(4).lower()[:180], b"", b"ACGT" * 7, b"N" * 40]
    for _ in range(300):
        n = rng.choice([rng.randint(0, 40), rng.randint(20, 256), rng.randint(250, 700)])
        seqs.append(bytes(rng.choice(alpha) for _ in range(n)))
    buf, offs = skq.pack_reads(seqs)
    s = skq.Session(gi, len(seqs), 700)
    d_buf = skq.DeviceBuffer.from_numpy(buf)
    d_offs = skq.DeviceBuffer.from_numpy(offs)
    s.sketch(d_buf.ptr, d_offs.ptr, len(seqs), 700, nthash=True)
    s.check()
    out = s.export()
    assert (out["status"] == 0).all()
    ho = out["hash_offs"]
    for r, q in enumerate(seqs):
        for i, k in enumerate(ks):
            e = r * len(ks) + i
            got = list(out["hashes"][ho[e]:ho[e + 1]])
            exp = orc.sketch(q, k) if len(q) >= k else []
            assert got == exp, (r, k, len(q))


@pytest.mark.parametrize("fraction", [0.0, 0.5, 0.9, 1.0, 1.5, -1.0])
def test_chain_fractions(tx300, fraction):
    gi, oi = build([21, 31], tx=tx300)
    bases, _, _ = synth.reads(tx300, 800, 150, seed=17, err=0.01)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(800)]
    out = run_gpu(gi, reads, fraction=fraction)
    ref = oi.map_batch(reads, fraction=fraction)
    compare(out, ref, len(reads), 2)


def test_wide_postings_take_slow_chain_path():
    # hand-built index: some hashes map to 40 transcripts (> DCAP distinct per read) and the
    # candidate list exceeds the 16 fixed slots
    rng = np.random.default_rng(0)
    ntx = 200
    reads_tx = synth.transcriptome(20, seed=8)
    seqs = [reads_tx.seq(t) for t in range(reads_tx.ntx)]
    h, t = [], []
    for tid, s in enumerate(seqs):
        for x in orc.sketch(s, 31):
            h.append(x)
            t.append(tid)
            if rng.random() < 0.3:
                for extra in rng.choice(np.arange(20, ntx), 40, replace=False):
                    h.append(x)
                    t.append(int(extra))
    pairs = [(np.array(h, np.uint32), np.array(t, np.uint32))]
    gi, oi = build([31], pairs=pairs, ntx=ntx)
    bases, _, _ = synth.reads(reads_tx, 400, 150, seed=9)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(400)]
    for fraction in (0.9, 0.0):
        out = run_gpu(gi, reads, fraction=fraction)
        ref = oi.map_batch(reads, fraction=fraction)
        compare(out, ref, len(reads), 1)
        assert ref["cand_cnt"].max() > 16 or fraction != 0.0


def test_slow_reads_past_the_wave_path():
    """Reads the map kernel lists go to the wave slow path (k_slow_wave) first; those past its
    limits go on to the general paths: > 255 retained hashes per k (fraction 0.9, 300 bp), > 256
    distinct transcripts (fraction 0.3 with every hash mapping to 40 transcripts), > 512 windows
    (600 bp). Mixed with ordinary slow reads in one batch."""
    rng = np.random.default_rng(11)
    ntx = 3000
    tx = synth.transcriptome(24, seed=12)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    thr = orc.threshold(0.3)
    h, t = [], []
    for tid, s in enumerate(seqs):
        for x in orc.sketch(s, 31, thr=orc.threshold(0.95)):
            h.append(x)
            t.append(tid)
            if rng.random() < 0.5:
                for extra in rng.choice(np.arange(24, ntx), 40, replace=False):
                    h.append(x)
                    t.append(int(extra))
    pairs = [(np.array(h, np.uint32), np.array(t, np.uint32))]
    gi, oi = build([31], pairs=pairs, ntx=ntx)
    long = [s for s in seqs if len(s) >= 700]
    assert long
    reads = []
    for i in range(300):
        s = seqs[i % len(seqs)]
        L = min(len(s), (150, 150, 300, 600)[i % 4])
        p = int(rng.integers(0, len(s) - L + 1))
        reads.append(s[p:p + L])
    for th, fraction in ((thr, 0.9), (thr, 0.0), (orc.threshold(0.9), 0.0)):
        out = run_gpu(gi, reads, thr=th, fraction=fraction)
        ref = oi.map_batch(reads, thr=th, fraction=fraction)
        compare(out, ref, len(reads), 1)
        assert fraction > 0 or int(ref["cand_cnt"].max()) > 256
        tr, ts = totals_from(ref, len(reads), ntx)
        np.testing.assert_array_equal(out["totals"][0], tr)
        np.testing.assert_array_equal(out["totals"][1], ts)


def test_long_read_at_the_maximal_threshold(tx300):
    """A read longer than the slow sketch path's LDS holds, with every window retained (threshold
    UINT32_MAX): its packed run needs the two header words past its windows (round-3 advice: the
    run was sized for the windows alone and the map failed with E_HASH_EXT)."""
    gi, oi = build([31], tx=tx300)
    rng = np.random.default_rng(5)
    long = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 5000))
    reads = [long, tx300.seq(0)[:150], long[:4200], tx300.seq(1)[:150]]
    thr = 0xFFFFFFFF
    out = run_gpu(gi, reads, thr=thr)
    ref = oi.map_batch(reads, thr=thr)
    compare(out, ref, len(reads), 1)


def test_list_lengths_around_the_inline_limit():
    # hand-built index whose lists hold 1..12 transcripts: wide entries keep 7 inline and read
    # the rest from the postings list; each read stays within 16 distinct transcripts (the
    # extras of one source transcript come from its own group of 11)
    rng = np.random.default_rng(5)
    src = synth.transcriptome(20, seed=15)
    seqs = [src.seq(t) for t in range(src.ntx)]
    ntx = 20 + 20 * 11
    h, t = [], []
    for tid, s in enumerate(seqs):
        group = 20 + 11 * tid + np.arange(11)
        for x in orc.sketch(s, 31):
            h.append(x)
            t.append(tid)
            for extra in rng.choice(group, int(rng.integers(0, 12)), replace=False):
                h.append(x)
                t.append(int(extra))
    pairs = [(np.array(h, np.uint32), np.array(t, np.uint32))]
    gi, oi = build([31], pairs=pairs, ntx=ntx)
    assert gi.stats()["max_list"] >= 10
    bases, _, _ = synth.reads(src, 600, 150, seed=16)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(600)]
    for fraction in (0.9, 0.0):
        out = run_gpu(gi, reads, fraction=fraction)
        ref = oi.map_batch(reads, fraction=fraction)
        compare(out, ref, len(reads), 1)


def test_crowded_blocks():
    # hand-built index: below each real key, up to 3 extra keys in its 32-key block (ranks 2+ of
    # a rank table's block take its overflow array), with lists of 1..9 transcripts
    rng = np.random.default_rng(6)
    src = synth.transcriptome(30, seed=18)
    seqs = [src.seq(t) for t in range(src.ntx)]
    ntx = 60
    h, t = [], []
    for tid, s in enumerate(seqs):
        for x in orc.sketch(s, 31):
            h.append(x)
            t.append(tid)
            low = x & 31
            for j in rng.choice(low, min(low, int(rng.integers(0, 4))), replace=False) if low else []:
                for extra in rng.choice(ntx, int(rng.integers(1, 10)), replace=False):
                    h.append((x & ~31) | int(j))
                    t.append(int(extra))
    pairs = [(np.array(h, np.uint32), np.array(t, np.uint32))]
    gi, oi = build([31], pairs=pairs, ntx=ntx)
    bases, _, _ = synth.reads(src, 500, 150, seed=19, err=0.01)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(500)]
    out = run_gpu(gi, reads)
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), 1)


def test_index_without_some_k():
    # k list [21, 31] but the index only holds k=31: k=21 is skipped (src/sparse_chaining.cpp:51-53)
    tx = synth.transcriptome(100, seed=12)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    buf, offs = skq.pack_reads(seqs)
    tabs = skq.build_tables(buf, offs, [31])
    gi = skq.Index([21, 31], len(seqs), tabs)
    keys, o, tids = tabs[31]
    cnt = np.diff(o.astype(np.int64))
    oi = orc.Index([21, 31], pairs=[(np.zeros(0, np.uint32), np.zeros(0, np.uint32)),
                                    (np.repeat(keys, cnt), tids)], ntx=len(seqs))
    bases, _, _ = synth.reads(tx, 300, 150, seed=2)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(300)]
    out = run_gpu(gi, reads)
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), 2)


def test_wide_transcript_ids_take_the_64bit_key_kernel():
    """ntx > 2^22: candidates are sorted with 64-bit keys (k_count); ids near the top of the
    range must come back intact."""
    rng = np.random.default_rng(8)
    ntx = (1 << 22) + 50
    tx = synth.transcriptome(60, seed=9)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    remap = np.array(sorted(rng.choice(ntx, size=len(seqs), replace=False)), np.uint32)
    remap[-3:] = [ntx - 3, ntx - 2, ntx - 1]
    oi0 = orc.Index([31], seqs=seqs)
    keys, offs, tids = oi0.csr(0)
    h = np.repeat(keys, np.diff(offs.astype(np.int64)))
    pairs = [(h, remap[tids])]
    gi, oi = build([31], pairs=pairs, ntx=ntx)
    bases, _, _ = synth.reads(tx, 300, 150, seed=10)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(300)]
    out = run_gpu(gi, reads)
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), 1)
    assert int(out["cand_tid"].max()) >= (1 << 22)


def test_chain_sketches_entry_point(tx300):
    gi, oi = build([21, 31], tx=tx300)
    bases, _, _ = synth.reads(tx300, 500, 150, seed=30)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(500)]
    ref = oi.map_batch(reads)
    n, nk = len(reads), 2
    flat, offs, cnt = [], [], []
    present = np.ones(n * nk, np.uint8)
    rng = np.random.default_rng(1)
    for r in range(n):
        for i in range(nk):
            offs.append(len(flat))
            hs = list(ref["hashes"][r, i, :ref["hash_cnt"][r, i]])
            if rng.random() < 0.1:
                present[r * nk + i] = 0
            cnt.append(len(hs))
            flat += hs
    flat = np.array(flat + [0], np.uint32)
    d_h = skq.DeviceBuffer.from_numpy(flat)
    d_o = skq.DeviceBuffer.from_numpy(np.array(offs, np.uint64))
    d_c = skq.DeviceBuffer.from_numpy(np.array(cnt, np.uint32))
    d_p = skq.DeviceBuffer.from_numpy(present)
    s = skq.Session(gi, n, 150)
    s.chain_sketches(n, d_h.ptr, d_o.ptr, d_c.ptr, d_p.ptr, fraction=0.9)
    s.check()
    out = s.export()
    import ctypes as C
    co = out["cand_offs"]
    for r in range(n):
        hp = [np.ascontiguousarray(ref["hashes"][r, i, :ref["hash_cnt"][r, i]], np.uint32) for i in range(nk)]
        arr = (C.c_void_p * nk)(*[x.ctypes.data for x in hp])
        nh = np.array([ref["hash_cnt"][r, i] for i in range(nk)], np.uint32)
        pres = np.array([present[r * nk + i] for i in range(nk)], np.int32)
        t = np.zeros(tx300.ntx, np.uint32)
        sc = np.zeros(tx300.ntx, np.uint32)
        c = orc.lib().orc_chain_read(oi.h, arr, orc.ptr(nh), orc.ptr(pres), 0.9, orc.ptr(t), orc.ptr(sc), tx300.ntx)
        assert list(out["cand_tid"][co[r]:co[r + 1]]) == list(t[:c])
        assert list(out["cand_score"][co[r]:co[r + 1]]) == list(sc[:c])


@pytest.mark.parametrize("n", [1000, 600_000, 4_200_000])
def test_repeated_batches_accumulate_totals(tx300, n, probe_mode):
    """Three different batches through one session, totals accumulated. n = 4.2M (>= 2^22 reads):
    a fused map's tail (slow paths, totals binning) runs on the session's side stream and
    consecutive batches alternate between the session's two frames, the next map writing one while
    the previous tail still reads and writes the other. The totals are the three batches' sums, and
    the results read after a batch are that batch's own, read by read (per-read digests: status,
    retained-hash sets, candidate lists; tests/digest.py)."""
    import digest
    if n > 1_000_000 and probe_mode != "chain":
        pytest.skip("the side-stream frames once, over the default index kind")
    gi, oi = build([31], tx=tx300)
    s = skq.Session(gi, n, 150)
    tr = np.zeros(tx300.ntx, np.uint64)
    ts = np.zeros(tx300.ntx, np.uint64)
    keep = []
    for b in range(3):
        bases, _, _ = synth.reads(tx300, n, 150, seed=44 + b)
        d = skq.DeviceBuffer.from_numpy(bases)
        keep.append(d)  # (freed at the end: a batch's tail may still read its reads)
        s.map(d.ptr, None, n, 150, fixed_len=150)
        cpu = orc.map_digest(oi, bases, 150, nthreads=16)
        tr += cpu["tx_reads"]
        ts += cpu["tx_score"]
        if b != 1:  # (batch 1's results are left unread: batch 2 resets its frame behind its tail)
            s.check()
            dg = digest.export_digest(s.export(), 1)
            bad = np.nonzero(dg != cpu["digest"])[0]
            assert len(bad) == 0, "batch %d: %d reads differ (first %s)" % (b, len(bad), bad[:8].tolist())
    a, c = s.totals()
    np.testing.assert_array_equal(a, tr)
    np.testing.assert_array_equal(c, ts)
    s.reset_totals()
    a, _ = s.totals()
    assert a.sum() == 0
    s.free()
    for d in keep:
        d.free()


def test_mixed_batch_sizes_switch_streams(tx300, probe_mode):
    """Batches of alternating size through one session, totals accumulated: 4.2M reads (tail on the
    side stream, the other frame), 1000 (tail on the launch stream, after waiting for the side
    stream), 4.2M (the fork behind a launch-stream tail), 600k, 4.2M, 4.2M. Each batch's results per
    read right after it, and the running totals after each, against the oracle — the hand-offs
    between the two streams and the two frames' control words in every order they occur."""
    import digest
    if probe_mode != "chain":
        pytest.skip("the streams and frames once, over the default index kind")
    gi, oi = build([31], tx=tx300)
    sizes = [4_200_000, 1000, 4_200_000, 600_000, 4_200_000, 4_200_000]
    s = skq.Session(gi, max(sizes), 150)
    tr = np.zeros(tx300.ntx, np.uint64)
    ts = np.zeros(tx300.ntx, np.uint64)
    keep = []
    for b, n in enumerate(sizes):
        bases, _, _ = synth.reads(tx300, n, 150, seed=90 + b)
        d = skq.DeviceBuffer.from_numpy(bases)
        keep.append(d)
        s.map(d.ptr, None, n, 150, fixed_len=150)
        cpu = orc.map_digest(oi, bases, 150, nthreads=16)
        tr += cpu["tx_reads"]
        ts += cpu["tx_score"]
        if b != 4:  # (batch 4's results are left unread: the next batch resets its frame behind its tail)
            s.check()
            dg = digest.export_digest(s.export(), 1)
            bad = np.nonzero(dg != cpu["digest"])[0]
            assert len(bad) == 0, "batch %d (%d reads): %d reads differ (first %s)" % (b, n, len(bad), bad[:8].tolist())
            a, c = s.totals()
            np.testing.assert_array_equal(a, tr, err_msg="after batch %d" % b)
            np.testing.assert_array_equal(c, ts, err_msg="after batch %d" % b)
    a, c = s.totals()
    np.testing.assert_array_equal(a, tr)
    np.testing.assert_array_equal(c, ts)
    s.free()
    for d in keep:
        d.free()


def test_very_long_reads_and_large_postings():
    # whole transcripts as reads (up to ~4 kb) plus 8-12 kb concatenations: the slow sketch path
    # beyond its LDS capacity and the slow chain path beyond LDS (global scratch)
    rng = np.random.default_rng(5)
    tx = synth.transcriptome(60, seed=77)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    h, t = [], []
    for tid, s in enumerate(seqs):
        for x in orc.sketch(s, 31):
            h.append(x)
            t.append(tid)
            if rng.random() < 0.5:
                for extra in rng.choice(np.arange(60, 400), 30, replace=False):
                    h.append(x)
                    t.append(int(extra))
    pairs = [(np.array(h, np.uint32), np.array(t, np.uint32))]
    gi, oi = build([31], pairs=pairs, ntx=400)
    reads = seqs[:20] + [b"".join(seqs[i:i + 4]) for i in range(0, 16, 4)]
    thr = orc.threshold(0.9)  # > SLOW_CAP retained hashes for the long ones
    for th in (None, thr):
        out = run_gpu(gi, reads, thr=th)
        ref = oi.map_batch(reads, thr=th)
        compare(out, ref, len(reads), 1)


def test_multi_k_general_slow_paths(tx300, probe_mode):
    """Multi-k batches whose slow reads reach the general paths behind k_slow_wave: reads longer
    than the wave path's 512 windows (re-sketched by k_general_slow, the ovf3 list) and more than
    255 retained hashes per k (a threshold near UINT32_MAX), mixed with ordinary reads of the same
    waves, so the re-sketch of one read runs while other workgroups chain reads whose packed offsets
    depend on it (run marks carry the region shares). Bit-exact per read and in the
    totals."""
    ks = [21, 25, 31]
    gi, oi = build(ks, tx=tx300)
    rng = random.Random(17)
    reads = []
    for i in range(700):
        s = b"".join(tx300.seq(rng.randrange(tx300.ntx)) for _ in range(3))
        L = rng.choice([150, 150, 150, 600, 900, 1500]) if i % 5 == 0 else 150
        L = min(L, len(s))
        p = rng.randint(0, len(s) - L)
        reads.append(bytes(s[p:p + L]))
    for th in (None, orc.threshold(0.6)):
        out = run_gpu(gi, reads, thr=th)
        ref = oi.map_batch(reads, thr=th)
        compare(out, ref, len(reads), len(ks))
        tr, ts = totals_from(ref, len(reads), tx300.ntx)
        np.testing.assert_array_equal(out["totals"][0], tr)
        np.testing.assert_array_equal(out["totals"][1], ts)


@pytest.mark.parametrize("ks,read_len", [([21, 25, 31], 150), ([31, 31], 150), ([25, 31], 100), ([21, 31], 220)])
def test_fused_multi_k_path_is_taken_and_exact(tx300, probe_mode, ks, read_len):
    """With wide or compact tables, 2-4 k slots map through the k slots' passes (one k_map1 launch
    each) with no separate count launch; every other probe structure through k_sketch + a count
    kernel. All bit-exact."""
    gi, oi = build(ks, tx=tx300)
    bases, _, _ = synth.reads(tx300, 2000, read_len, seed=77, err=0.002)
    reads = [bases[i * read_len:(i + 1) * read_len].tobytes() for i in range(2000)]
    buf, offs = skq.pack_reads(reads)
    s = skq.Session(gi, len(reads), read_len)
    d_buf = skq.DeviceBuffer.from_numpy(buf)
    s.enable_timing(True)
    if SPLIT:
        s.sketch(d_buf.ptr, None, len(reads), read_len, fixed_len=read_len)
        s.chain()
    else:
        s.map(d_buf.ptr, None, len(reads), read_len, fixed_len=read_len)
    s.check()
    s.enable_timing(False)
    count_launches = s.kernel_time(2)[1]
    if probe_mode in ("wide", "compact", "chain", "chain-compact"):
        assert count_launches == 0 and s.kernel_time(0)[1] == 1
    else:
        assert count_launches == 1
    out = s.export()
    out["totals"] = s.totals()
    ref = oi.map_batch(reads)
    compare(out, ref, len(reads), len(ks))
    tr, ts = totals_from(ref, len(reads), tx300.ntx)
    np.testing.assert_array_equal(out["totals"][0], tr)
    np.testing.assert_array_equal(out["totals"][1], ts)


def test_multi_k_passes_base_image(tx300, probe_mode):
    """The k_map1 passes: the first stores each wave's staged bases (2-bit codes + bad bits) and
    the later passes stage from that image. Variable lengths, an unaligned buffer, bad bytes, short
    and > 256-bp reads and several batches through one session (the image grows with the batch):
    bit-exact."""
    ks = [21, 25, 31]
    gi, oi = build(ks, tx=tx300)
    rng = random.Random(11)
    reads = []
    for i in range(2500):
        s = tx300.seq(rng.randrange(tx300.ntx))
        L = rng.choice([0, 20, 31, 90, 150, 150, 150, 199, 256, 300]) if i % 3 else rng.randint(0, 260)
        L = min(L, len(s))
        p = rng.randint(0, len(s) - L)
        r = bytearray(s[p:p + L])
        if L and i % 97 == 0:
            r[rng.randrange(L)] = ord("N")
        reads.append(bytes(r))
    ref = oi.map_batch(reads)
    s = skq.Session(gi, 1500, 300)
    for lo, hi in ((1500, 2500), (0, 1500), (0, 1000)):  # (the image grows, then a smaller batch)
        buf, offs = skq.pack_reads(reads[lo:hi])
        pad = np.concatenate([np.zeros(5, np.uint8), buf])  # reads start 5 bytes into the buffer
        d_buf = skq.DeviceBuffer.from_numpy(pad)
        d_offs = skq.DeviceBuffer.from_numpy(offs)
        at = C.c_void_p(d_buf.value + 5)
        if SPLIT:
            s.sketch(at, d_offs.ptr, hi - lo, 300)
            s.chain()
        else:
            s.map(at, d_offs.ptr, hi - lo, 300)
        s.check()
        out = s.export()
        sub = {key: v[lo:hi] for key, v in ref.items()}
        compare(out, sub, hi - lo, len(ks))
