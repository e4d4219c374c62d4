"""The totals binning's rare paths (k_bin_packed<4096, 4>, launch_bin): a transcript set of groups
of twelve near-copies, so every read lists ~12 candidates — a map wave's packed region then holds
more than the 256 words loaded with the counts (the words past 256 are re-read per lane), and four
map workgroups more than the 4096 words the staging holds (their candidates go straight into the
totals with 64-bit atomics). > 32768 transcripts, so the totals take the grouped binning (5
buckets of 2^13 ids). Per read (digest) and per transcript against the oracle."""
import numpy as np
import pytest
import torch  # noqa: F401  (one HIP runtime per process)

import digest
import orc
import skq
from skq import synth

pytestmark = pytest.mark.gpu

L, N, COPIES, BASE = 150, 300_000, 12, 3_400


def _copies_transcriptome(seed=71):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    pieces, names = [], []
    for b in range(BASE):
        s = acgt[rng.integers(0, 4, int(rng.integers(400, 1500)))]
        for c in range(COPIES):
            x = s.copy()
            x[rng.integers(0, len(x), 2)] = acgt[rng.integers(0, 4, 2)]  # (two substitutions per copy)
            pieces.append(x)
            names.append("COPY%05d-%02d" % (b, c))
    lens = np.array([len(p) for p in pieces], np.uint64)
    offs = np.zeros(len(pieces) + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    return synth.Transcriptome(np.concatenate(pieces), offs, names)


def test_binning_overflow_paths_match_the_oracle():
    tx = _copies_transcriptome()
    assert tx.ntx > 32768
    ks = [31]
    tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
    keys, offs, tids = tables[31]
    oi = orc.Index(ks, pairs=[(np.repeat(keys, np.diff(offs.astype(np.int64))), tids)], ntx=tx.ntx)
    bases, _, _ = synth.reads(tx, N, L, seed=72, err=0.001)
    cpu = orc.map_digest(oi, bases, L, nthreads=16)
    d = skq.DeviceBuffer.from_numpy(bases)
    for chained in (False, True):
        index = skq.Index(ks, tx.ntx, tables, seqs=(tx.seqs, tx.offs) if chained else None)
        s = skq.Session(index, N, L)
        s.map(d.ptr, None, N, L, fixed_len=L)
        s.check()
        out = s.export()
        tot = s.totals()
        dg = digest.export_digest(out, len(ks))
        s.free()
        index.free()
        per_read = np.diff(out["cand_offs"].astype(np.int64))
        assert per_read.mean() > 6, per_read.mean()  # (the overflow paths are taken)
        bad = np.nonzero(dg != cpu["digest"])[0]
        assert len(bad) == 0, "chained=%s: %d reads differ (first %s)" % (chained, len(bad), bad[:8].tolist())
        np.testing.assert_array_equal(tot[0], cpu["tx_reads"])
        np.testing.assert_array_equal(tot[1], cpu["tx_score"])
    d.free()
