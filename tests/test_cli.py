"""The skq command line end to end on the GPU (index -> quant -> CSV): the SURVEY §8c edge
fixture's expected rows, and a synthetic run with duplicated, invalid and short reads compared
with the oracle pipeline (record rules restated here, oracle sparse chain, oracle EM)."""
import os
import random
import subprocess

import numpy as np
import pytest

import orc
from skq import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EDGE = os.path.join(ROOT, "tests", "golden", "edge")
CLI = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "skq")


def run(*args, env=None):
    return subprocess.run([CLI, *map(str, args)], check=True, capture_output=True, text=True, timeout=300,
                          env=env).stdout


def rows(path):
    lines = open(path).read().splitlines()
    assert lines[0] == "Name,NumReads,EM_Abundance"
    return {tuple(l.split(",")) for l in lines[1:]}


def test_edge_fixture(tmp_path):
    idx, csv = tmp_path / "e.idx", tmp_path / "e.csv"
    out = run("-k", "31", "-o", "index", os.path.join(EDGE, "e.fa"), idx)
    assert "Index built in" in out and "Index saved to" in out
    out = run("-o", "quant", idx, os.path.join(EDGE, "e.fq"), csv)
    for msg in ("Loading index completed", "Loading read completed", "Sparse chaining completed",
                "EM estimation completed", "Read assignment completed", "Output written to"):
        assert msg in out
    assert rows(csv) == {("T2", "2", "2.01333"), ("T4last", "1", "1.01333")}


def test_quant_uses_the_index_k_list(tmp_path):
    # -k at quant time is ignored: load_index overwrites the list (src/main.cpp:172-178)
    idx, a, b = tmp_path / "e.idx", tmp_path / "a.csv", tmp_path / "b.csv"
    run("-k", "31", "-o", "index", os.path.join(EDGE, "e.fa"), idx)
    run("-o", "quant", idx, os.path.join(EDGE, "e.fq"), a)
    run("-k", "21,25", "-o", "quant", idx, os.path.join(EDGE, "e.fq"), b)
    assert rows(a) == rows(b)


def _records(path):
    """process_fastq_single_pass's reader restated (src/main.cpp:120-147)."""
    lines = open(path, "rb").read().split(b"\n")
    recs, i = [], 0
    while i < len(lines):
        line = lines[i]
        i += 1
        if not line or line[:1] != b"@":
            continue
        seq = lines[i] if i < len(lines) else b""
        i += 3
        recs.append((line[1:], seq))
    return recs


@pytest.mark.parametrize("ks,devices", [([31], None), ([21, 25, 31], None), ([31], "0,0"), ([21, 25, 31], "0,0,0")])
def test_synthetic_quant_matches_the_oracle_pipeline(tmp_path, ks, devices):
    """devices: SKQ_DEVICES, the file split in parts mapped by one host thread and device index
    each (here the same GPU several times: the posterior sums reduce through the host instead of
    RCCL), duplicate ids settled across the parts, EM rounds sharded over the parts."""
    tx = synth.transcriptome(150, seed=61)
    fa, fq = tmp_path / "t.fa", tmp_path / "r.fq"
    tx.write_fasta(fa)
    bases, tids, starts = synth.reads(tx, 3000, 150, seed=62)
    reads = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(3000)]
    rng = random.Random(63)
    recs = [(b"read%d" % i, r) for i, r in enumerate(reads)]
    for i in rng.sample(range(3000), 60):   # invalid bases, lowercase, short reads
        s = recs[i][1]
        recs[i] = (recs[i][0], rng.choice([s[:70] + b"N" + s[71:], s.lower(), s[:25]]))
    for i in rng.sample(range(3000), 80):   # duplicate ids later in the file (valid or not)
        j = rng.randrange(3000)
        recs.append((recs[i][0], rng.choice([reads[j], reads[j][:10]])))
    with open(fq, "wb") as f:
        for name, s in recs:
            f.write(b"@" + name + b"\n" + s + b"\n+\n" + b"I" * len(s) + b"\n")
    idx, csv = tmp_path / "t.idx", tmp_path / "t.csv"
    run("-k", ",".join(map(str, ks)), "-o", "index", fa, idx)
    env = dict(os.environ, SKQ_BATCH="700")  # several batches
    if devices:
        env["SKQ_DEVICES"] = devices
    run("-o", "quant", idx, fq, csv, env=env)

    # oracle pipeline
    names = [n.encode() for n in tx.names]
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    last = {}
    for o, (name, s) in enumerate(_records(fq)):
        if all(c in b"ACGT" for c in s) and len(s) >= max(ks):
            last[name] = o
    kept = [s for o, (name, s) in enumerate(_records(fq)) if last.get(name) == o]
    ref = orc.Index(ks, seqs=seqs).map_batch(kept)
    offs = np.concatenate([[0], np.cumsum(ref["cand_cnt"])]).astype(np.uint64)
    ct = np.concatenate([ref["cand_tid"][r, :ref["cand_cnt"][r]] for r in range(len(kept))]).astype(np.uint32)
    cs = np.concatenate([ref["cand_score"][r, :ref["cand_cnt"][r]] for r in range(len(kept))]).astype(np.uint32)
    pi, _ = orc.em(offs, ct, cs, tx.ntx)
    counts, assigned = orc.assign(offs, ct, cs, tx.ntx, pi)
    exp = {names[t].decode(): (counts[t], pi[t]) for t in range(tx.ntx) if assigned[t]}
    got = {r[0]: (float(r[1]), float(r[2])) for r in rows(csv)}
    assert set(got) == set(exp) and len(got) > 100
    for n, (c, p) in exp.items():  # printed with 6 significant digits
        assert got[n][0] == pytest.approx(float("%g" % c), rel=2e-6, abs=1e-12), n
        assert got[n][1] == pytest.approx(float("%g" % p), rel=2e-6), n
