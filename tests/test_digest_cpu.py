"""The per-read digest (oracle/oracle.c orc_map_digest) and its numpy restatement over an export
(tests/digest.py) agree read by read on the oracle's own per-read outputs, and the digest changes
when one read's result changes — what lets the GPU tests compare per-read results at full batch
sizes (tests/test_gpu_scale.py test_full_batch_totals)."""
import numpy as np

import digest
import orc
from skq import synth


def _export_of(ref, nk):
    """orc_map_batch outputs in the layout of skq Session.export()."""
    n = len(ref["status"])
    hc = ref["hash_cnt"].astype(np.int64)  # [n, nk]
    ho = np.zeros(n * nk + 1, np.uint64)
    ho[1:] = np.cumsum(hc.reshape(-1))
    hcap = ref["hashes"].shape[2]
    hm = np.arange(hcap)[None, None, :] < hc[:, :, None]
    co = np.zeros(n + 1, np.uint64)
    co[1:] = np.cumsum(ref["cand_cnt"].astype(np.int64))
    ccap = ref["cand_tid"].shape[1]
    cm = np.arange(ccap)[None, :] < ref["cand_cnt"][:, None]
    return dict(status=ref["status"], hash_offs=ho, hashes=ref["hashes"][hm], cand_offs=co,
                cand_tid=ref["cand_tid"][cm], cand_score=ref["cand_score"][cm])


def test_digest_matches_numpy_restatement_and_detects_changes():
    tx = synth.transcriptome(400, seed=7)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    ks = [21, 31]
    oi = orc.Index(ks, seqs=seqs)
    L, n = 150, 3000
    bases, _, _ = synth.reads(tx, n, L, seed=8, err=0.002)
    bases[L * 5 + 9] = ord("N")  # an invalid read
    bases[L * 11] = ord("a")     # a lowercase one
    reads = [bases[i * L:(i + 1) * L].tobytes() for i in range(n)]
    ref = oi.map_batch(reads, hcap=L, ccap=oi.ntx)
    a = orc.map_digest(oi, bases, L, nthreads=3)
    b = orc.map_digest(oi, bases, L, nthreads=1, totals=False)
    np.testing.assert_array_equal(a["digest"], b["digest"])
    ex = _export_of(ref, len(ks))
    d = digest.export_digest(ex, len(ks))
    np.testing.assert_array_equal(d, a["digest"])
    assert len(np.unique(d)) > 0.9 * n
    # totals from the per-read lists
    tr = np.zeros(oi.ntx, np.uint64)
    ts = np.zeros(oi.ntx, np.uint64)
    cm = np.arange(ref["cand_tid"].shape[1])[None, :] < ref["cand_cnt"][:, None]
    np.add.at(tr, ref["cand_tid"][cm], 1)
    np.add.at(ts, ref["cand_tid"][cm], ref["cand_score"][cm].astype(np.uint64))
    np.testing.assert_array_equal(a["tx_reads"], tr)
    np.testing.assert_array_equal(a["tx_score"], ts)
    # a candidate list moved to the next read keeps the totals but not the digests
    r = int(np.nonzero(ref["cand_cnt"] > 1)[0][0])
    ex2 = dict(ex)
    co = ex["cand_offs"].astype(np.int64)
    co2 = co.copy()
    co2[r + 1] -= 1  # read r's last candidate becomes read r + 1's first
    ex2["cand_offs"] = co2.astype(np.uint64)
    d2 = digest.export_digest(ex2, len(ks))
    assert (d2 != d).sum() == 2 and d2[r] != d[r] and d2[r + 1] != d[r + 1]
    # two equal-score candidates swapped inside one read
    ex3 = dict(ex)
    ct = ex["cand_tid"].copy()
    s0 = int(co[r])
    ct[s0], ct[s0 + 1] = ct[s0 + 1], ct[s0]
    ex3["cand_tid"] = ct
    assert (digest.export_digest(ex3, len(ks)) != d).sum() == 1
