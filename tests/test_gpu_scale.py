"""GPU parity at BASELINE.json's scales (cfg2, cfg3, cfg5), through the C ABI, bit-exact against
the CPU oracle run over the same reads as FASTQ text (orc_fastq_map, threads over read shards).

  cfg2: 10k-transcript index, 100 bp reads, k = 31;
  cfg3: ~200k-transcript GENCODE-scale index, 150 bp, k = 31 (the metric's config);
  cfg5: the same index at k = {21, 25, 31} (the fused multi-k map).

Per read: status, retained-hash sets per k, candidate lists (tid, score; score desc, tid asc);
per transcript: candidate reads and summed scores. cfg3 is also checked at its FULL batch
(10M reads) through the size-independent per-transcript totals, which exercise the slow paths,
the overflow lists and the per-batch totals packing at the bench's own size.
"""
import os

import numpy as np
import pytest
import torch  # noqa: F401  (before skq: one HIP runtime per process)

import orc
import skq
from skq import synth

pytestmark = pytest.mark.gpu

NTHREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def tx200k():
    return synth.transcriptome(200_000, seed=1)  # bench.py's cfg3 / cfg5 transcriptome


@pytest.fixture(scope="module")
def tx10k():
    return synth.transcriptome(10_000, seed=1)


def _oracle(tables, ks, ntx):
    pairs = []
    for k in ks:
        keys, offs, tids = tables[k]
        pairs.append((np.repeat(keys, np.diff(offs.astype(np.int64))), tids))
    return orc.Index(ks, pairs=pairs, ntx=ntx)


def _gpu_map(index, bases, n, L):
    s = skq.Session(index, n, L)
    d = skq.DeviceBuffer.from_numpy(bases[:n * L])
    s.map(d.ptr, None, n, L, fixed_len=L)
    s.check()
    out = s.export()
    tot = s.totals()
    slow = s.slow_reads()
    s.free()
    d.free()
    return out, tot, slow


def _compare(out, tot, cpu, nk):
    n = cpu["n"]
    np.testing.assert_array_equal(out["status"], cpu["status"])
    ho = out["hash_offs"].astype(np.int64)
    np.testing.assert_array_equal(np.diff(ho).reshape(n, nk), cpu["hash_cnt"].astype(np.int64))
    hcap = cpu["hashes"].shape[2]
    hm = np.arange(hcap)[None, None, :] < cpu["hash_cnt"][:, :, None]
    np.testing.assert_array_equal(out["hashes"][:ho[-1]], cpu["hashes"][hm])
    co = out["cand_offs"].astype(np.int64)
    np.testing.assert_array_equal(np.diff(co), cpu["cand_cnt"].astype(np.int64))
    ccap = cpu["cand_tid"].shape[1]
    cm = np.arange(ccap)[None, :] < cpu["cand_cnt"][:, None]
    np.testing.assert_array_equal(out["cand_tid"][:co[-1]], cpu["cand_tid"][cm])
    np.testing.assert_array_equal(out["cand_score"][:co[-1]], cpu["cand_score"][cm])
    np.testing.assert_array_equal(tot[0], cpu["tx_reads"])
    np.testing.assert_array_equal(tot[1], cpu["tx_score"])


def _case(tx, ks, L, nreads, seed, err=0.001, chained=False):
    tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=NTHREADS)
    index = skq.Index(ks, tx.ntx, tables, seqs=(tx.seqs, tx.offs) if chained else None)
    bases, _, _ = synth.reads(tx, nreads, L, seed=seed, err=err)
    # a sprinkle of edge reads at scale: invalid bases and lowercase
    rng = np.random.default_rng(seed)
    bad = rng.choice(nreads, nreads // 1000, replace=False)
    bases[bad * L + rng.integers(0, L, len(bad))] = ord("N")
    low = rng.choice(nreads, nreads // 2000, replace=False)
    bases[low * L] = ord("a")
    out, tot, slow = _gpu_map(index, bases, nreads, L)
    cpu = orc.fastq_map(_oracle(tables, ks, tx.ntx), synth.fastq_bytes(bases, L), nthreads=NTHREADS,
                        hcap=64, ccap=64)
    assert cpu["n"] == nreads
    _compare(out, tot, cpu, len(ks))
    st = index.stats()
    index.free()
    return cpu, st, slow


@pytest.mark.parametrize("mode", ["map1", "chain", "chain-compact", "chain-tight"])
def test_cfg2_10k_transcripts_100bp(tx10k, mode, monkeypatch):
    """chain-compact: the chained tables at the compact tables' slots (SKQ_CHAIN=2); chain-tight: a
    device budget the chained tables per possible key do not fit (SKQ_CHAIN_MB=2048), so the index
    sizes itself to compact entries + chained tables per present key."""
    monkeypatch.setenv("SKQ_CHAIN", "0" if mode == "map1" else "2" if mode == "chain-compact" else "1")
    if mode == "chain-tight":
        monkeypatch.setenv("SKQ_CHAIN_MB", "2048")
    cpu, st, _ = _case(tx10k, [31], 100, 300_000, seed=201, chained=mode != "map1")
    assert (cpu["cand_cnt"] > 0).mean() > 0.9
    assert st["probe"] in ("compact", "wide", "hash")
    if mode != "map1":
        assert st["chained"] > 2, st
        assert (st["probe"] == "compact") == (mode in ("chain-compact", "chain-tight")), st
        if st["probe"] == "compact":
            assert st["device_bytes"] < 2e9, st


@pytest.mark.parametrize("mode", ["map1", "chain", "chain-compact"])
def test_cfg3_200k_transcripts_150bp(tx200k, mode, monkeypatch):
    """chain: k_map1 over the chained tables (SKQ_CHAIN=1); chain-compact: over compact tables
    (SKQ_CHAIN=2)."""
    monkeypatch.setenv("SKQ_CHAIN", "0" if mode == "map1" else "2" if mode == "chain-compact" else "1")
    cpu, st, slow = _case(tx200k, [31], 150, 400_000, seed=301, chained=mode != "map1")
    assert (st["chained"] > 2) == (mode != "map1"), st
    assert (st["probe"] == "compact") == (mode == "chain-compact"), st
    assert (cpu["cand_cnt"] > 0).mean() > 0.95
    assert st["max_list"] >= 10  # GENCODE-scale postings (long lists take the inline overflow)
    assert slow[0] + slow[1] > 0  # the slow paths ran at scale and agreed


@pytest.mark.parametrize("mode", ["map1", "chain", "chain-compact"])
def test_cfg5_multi_k_200k_transcripts(tx200k, mode, monkeypatch):
    """chain: every k slot's pass over its own chained tables (3 x 27.5 GB), one k_map1 launch
    each; chain-compact: the chained entries at the compact slots (SKQ_CHAIN=2, 3 x ~0.6 GB)."""
    monkeypatch.setenv("SKQ_CHAIN", "0" if mode == "map1" else "2" if mode == "chain-compact" else "1")
    cpu, st, sl = _case(tx200k, [21, 25, 31], 150, 250_000, seed=501, chained=mode != "map1")
    assert (st["chained"] > 2) == (mode != "map1"), st
    assert (cpu["cand_cnt"] > 0).mean() > 0.95
    assert sl[0] > 100  # the k = 21 pass's capacity sends reads to the slow path


@pytest.mark.parametrize("n,seed,ks", [(10_000_000, 1000, [31]), (12_500_000, 1003, [31]), (10_000_000, 1000, [21, 25, 31])],
                         ids=["cfg3_10M", "cfg4_rank3_12.5M", "cfg5_10M"])
def test_full_batch_totals(tx200k, n, seed, ks, monkeypatch):
    """The bench's own batches, one skq_map each: cfg3 (10M x 150 bp, rank 0), cfg4's per-GPU
    shard (12.5M x 150 bp; rank 3's seed, as bench.py --gpus 8 draws it) and cfg5's batch (10M,
    multi-k passes, ~37k slow reads whose runs the slow wave writes while it reads other reads'
    packed offsets): per-transcript totals AND every read's own result equal the oracle's over the
    same reads. Per read: a 64-bit digest of its status, its retained-hash sets and its candidate
    list (oracle/oracle.c orc_map_digest; tests/digest.py over the export), so a candidate list
    moved between reads or equal-score entries swapped, which keep the totals, still fail
    (src/sparse_chaining.cpp:107-111: the reference's output is per read). Each batch runs three
    times against one oracle pass: over the wide entries, over the chained tables the bench and the
    CLI default to (an index given the transcripts' sequences), whose marker entries (lists > 8
    ids), queries past the table, slow-read hand-off and totals binning are then checked at the
    full batch too, and over the chained entries at the compact tables' slots (SKQ_CHAIN=2), where a
    query that is no key lands on another key's slot."""
    import digest
    L = 150
    tables = skq.build_tables(tx200k.seqs, tx200k.offs, ks, nthreads=NTHREADS)
    bases, _, _ = synth.reads(tx200k, n, L, seed=seed, err=0.001)  # bench.py's batch of rank seed - 1000
    cpu = orc.map_digest(_oracle(tables, ks, tx200k.ntx), bases, L, nthreads=NTHREADS)
    assert cpu["n"] == n
    d = skq.DeviceBuffer.from_numpy(bases)
    del bases
    for chained in (0, 1, 2):
        monkeypatch.setenv("SKQ_CHAIN", str(max(chained, 1)))
        index = skq.Index(ks, tx200k.ntx, tables, seqs=(tx200k.seqs, tx200k.offs) if chained else None)
        st = index.stats()
        assert (st["chained"] > 2) == bool(chained), st  # (1 + the mean records per entry; 0: none)
        assert (st["probe"] == "compact") == (chained == 2), st
        s = skq.Session(index, n, L)
        s.map(d.ptr, None, n, L, fixed_len=L)
        s.check()
        tot = s.totals()
        slow = s.slow_reads()
        dg = digest.export_digest(s.export(), len(ks))
        s.free()
        index.free()
        np.testing.assert_array_equal(tot[0], cpu["tx_reads"], err_msg="chained=%s" % chained)
        np.testing.assert_array_equal(tot[1], cpu["tx_score"], err_msg="chained=%s" % chained)
        bad = np.nonzero(dg != cpu["digest"])[0]
        assert len(bad) == 0, "chained=%s: %d reads differ (first %s)" % (chained, len(bad), bad[:8].tolist())
        assert int(tot[0].sum()) > 3 * n  # ~3.1 candidates per read
        assert slow[0] + slow[1] > 100
    d.free()
