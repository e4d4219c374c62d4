"""The totals' rare paths: a transcript set of groups of twelve near-copies, so every read lists
~12 candidates and a map wave's packed region holds more than the 256 words the totals kernels
load in their first round (the words past 256 are read again per lane). 3,400 groups (40,800
transcripts): the grouped binning (k_bin_packed<4096, 4>, 5 buckets of 2^13 ids), where four map
workgroups also overflow the 4096-word staging (their candidates go straight into the totals with
64-bit atomics). 1,000 groups (12,000 transcripts): k_tot_small, between the maps (300k reads) and
beside the next map on the side stream (4.2M reads, 256-thread workgroups, 4096-id ranges). Per
read (digest) and per transcript against the oracle."""
import numpy as np
import pytest
import torch  # noqa: F401  (one HIP runtime per process)

import digest
import orc
import skq
from skq import synth

pytestmark = pytest.mark.gpu

L, COPIES = 150, 12


def _copies_transcriptome(BASE, seed=71):
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


@pytest.mark.parametrize("base,N,modes", [(3_400, 300_000, (False, True)), (1_000, 300_000, (False, True)),
                                          (1_000, 4_200_000, (False,))],
                         ids=["grouped-bins", "tot-small", "tot-small-side"])
def test_binning_overflow_paths_match_the_oracle(base, N, modes):
    tx = _copies_transcriptome(base)
    assert (tx.ntx > 32768) == (base == 3_400) and (tx.ntx <= 16384) == (base == 1_000)
    ks = [31]
    tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
    keys, offs, tids = tables[31]
    oi = orc.Index(ks, pairs=[(np.repeat(keys, np.diff(offs.astype(np.int64))), tids)], ntx=tx.ntx)
    bases, _, _ = synth.reads(tx, N, L, seed=72, err=0.001)
    cpu = orc.map_digest(oi, bases, L, nthreads=16)
    d = skq.DeviceBuffer.from_numpy(bases)
    for chained in modes:
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
