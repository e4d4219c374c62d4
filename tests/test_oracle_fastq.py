"""The oracle's FASTQ-bytes path (orc_fastq_map: bench.py's CPU baseline and parity sample) agrees
with its per-read path and with the reference's record rules; threads change nothing."""
import os

import numpy as np

import orc
from skq import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EDGE = os.path.join(ROOT, "tests", "golden", "edge")


def test_edge_fastq_record_rules():
    names_seqs = open(os.path.join(EDGE, "e.fa"), "rb").read()
    tx = []
    for rec in names_seqs.split(b">")[1:]:
        lines = rec.split(b"\n")
        tx.append(b"".join(lines[1:]))
    oi = orc.Index([31], seqs=tx)
    fq = open(os.path.join(EDGE, "e.fq"), "rb").read()
    out = orc.fastq_map(oi, fq, nthreads=2)
    assert out["n"] == 8
    # r1's second record wins; r3 (N), r4 (short), r5 (lowercase), r7 (\r) are dropped
    assert list(np.nonzero(out["kept"])[0]) == [1, 5, 6]
    assert list(out["status"]) == [0, 0, 1, 2, 1, 0, 0, 1]  # ok / invalid / short


def test_fastq_path_equals_per_read_path_and_threads_agree():
    tx = synth.transcriptome(300, seed=3)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    oi = orc.Index([21, 31], seqs=seqs)
    bases, _, _ = synth.reads(tx, 4000, 150, seed=4, err=0.002)
    bases[150 * 7 + 3] = ord("N")  # one invalid read
    fq = synth.fastq_bytes(bases, 150)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(4000)]
    ref = oi.map_batch(reads, hcap=32, ccap=oi.ntx)
    a = orc.fastq_map(oi, fq, nthreads=1)
    b = orc.fastq_map(oi, fq, nthreads=7)
    c = orc.fastq_map(oi, fq, nthreads=5, outputs=False)
    assert a["n"] == b["n"] == c["n"] == 4000
    for k in ("status", "hash_cnt", "hashes", "cand_cnt", "cand_tid", "cand_score"):
        np.testing.assert_array_equal(a[k], ref[k])
        np.testing.assert_array_equal(b[k], ref[k])
    assert a["status"][7] == 1 and not a["kept"][7] and a["kept"].sum() == 3999
    tr = np.zeros(oi.ntx, np.uint64)
    ts = np.zeros(oi.ntx, np.uint64)
    for r in range(4000):
        if a["kept"][r]:
            for j in range(int(a["cand_cnt"][r])):
                tr[a["cand_tid"][r, j]] += 1
                ts[a["cand_tid"][r, j]] += a["cand_score"][r, j]
    for o in (a, b, c):
        np.testing.assert_array_equal(o["tx_reads"], tr)
        np.testing.assert_array_equal(o["tx_score"], ts)


def test_duplicate_ids_keep_the_last_valid_record():
    tx = synth.transcriptome(50, seed=8)
    oi = orc.Index([31], seqs=[tx.seq(t) for t in range(tx.ntx)])
    bases, _, _ = synth.reads(tx, 3, 150, seed=9)
    s = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(3)]
    q = b"I" * 150
    fq = (b"@x\n" + s[0] + b"\n+\n" + q + b"\n" + b"@y\n" + s[1] + b"\n+\n" + q + b"\n" +
          b"@x\n" + s[2] + b"\n+\n" + q + b"\n" + b"@x\n" + s[1][:-1] + b"N\n+\n" + q + b"\n")
    out = orc.fastq_map(oi, fq, nthreads=2)
    assert out["n"] == 4 and list(out["kept"]) == [False, True, True, False]
