"""The C++ drop-in against the reference's OWN call sites: src/main.cpp compiled unmodified with
include/dropin ahead of the reference's include/ and linked against libskq.so (oracle/ref.mk:
ref_cli_skq keeps the reference's data_io.cpp / isoform_assignment.cpp, ref_cli_skq_all takes
everything but main.cpp from libskq), plus the <nthash/nthash.hpp> that main.cpp includes
(include/dropin/nthash/nthash.hpp) pinned against ntHash's own tables.

CPU: the header against the tables and SURVEY.md §8c known answers; the reference CLI builds and
links (only where /root/reference exists: the binaries are test-only and git-ignored).
GPU: the reference CLI over libskq runs index + quant on the §8c edge fixture (exact rows) and on a
synthetic transcriptome, where its CSV agrees with the skq CLI's, across each other's index files."""
import os
import random
import subprocess

import pytest

from skq import synth
from test_oracle_golden import CONV, S2, table_forward_hash

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
EDGE = os.path.join(ROOT, "tests", "golden", "edge")
CLIS = [os.path.join(ROOT, "oracle", "_ref", n) for n in ("ref_cli_skq", "ref_cli_skq_all")]
SKQ = os.path.join(ROOT, "sketch-for-rna-seq_amd", "lib", "skq")

PROBE = r"""
#include <nthash/nthash.hpp>
#include <cstdio>
#include <iostream>
#include <string>
int main() {
    std::string seq;
    unsigned k;
    while (std::cin >> k >> seq) {
        nthash::NtHash h(seq, 1, (uint16_t)k);
        while (h.roll()) std::printf("%zu:%016llx ", h.get_pos(), (unsigned long long)h.get_forward_hash());
        std::printf("\n");
    }
}
"""


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("nth")
    src, exe = d / "probe.cpp", d / "probe"
    src.write_text(PROBE)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include", "dropin"), str(src), "-o", str(exe)],
                   check=True)
    return str(exe)


def run_probe(exe, cases):
    out = subprocess.run([exe], input="".join("%d %s\n" % (k, s.decode()) for k, s in cases), capture_output=True,
                         text=True, check=True).stdout.splitlines()
    res = []
    for line in out:
        pairs = [x.split(":") for x in line.split()]
        res.append(([int(p) for p, _ in pairs], [int(h, 16) for _, h in pairs]))
    return res


def test_nthash_header_known_answers(probe):
    (p1, h1), (p2, h2), (p3, h3) = run_probe(probe, [(31, b"ACGT" * 8), (31, b"A" * 31), (31, S2)])
    assert h1 == [0xA11AB471672CE8D2, 0x57EBDAA5E0CA14EE] and p1 == [0, 1]
    assert h2 == [0xFFFFFFFEAF928327]
    assert [h & 0xFFFFFFFF for h in h3[:3]] == [2113525738, 1496400953, 3048415779]
    assert sorted({h & 0xFFFFFFFF for h in h3 if (h & 0xFFFFFFFF) <= 214748367}) == [
        6901433, 28017476, 62078630, 110941329, 117651234, 183192842]


@pytest.mark.parametrize("k", [1, 3, 4, 5, 21, 25, 31, 32, 33, 63, 64, 65])
def test_nthash_header_matches_the_binarys_tables(probe, k):
    rng = random.Random(7 * k)
    cases = []
    for _ in range(8):
        s = bytearray(rng.choice(b"ACGTacgtUu") for _ in range(rng.randint(k, k + 150)))
        for _ in range(rng.randint(0, 3)):
            s[rng.randrange(len(s))] = rng.choice(b"NnX-")
        cases.append((k, bytes(s)))
    for (k, s), (pos, hs) in zip(cases, run_probe(probe, cases)):
        expect = [j for j in range(len(s) - k + 1) if all(CONV[c] != 255 for c in s[j:j + k])]
        assert pos == expect
        assert hs == [table_forward_hash(s[j:j + k], k) for j in expect]


def test_nthash_header_argument_errors(probe):
    r = subprocess.run([probe], input="31 ACGT\n", capture_output=True, text=True)
    assert r.returncode != 0 and "[ntHash::NtHash] ERROR: sequence length (4) is smaller than k (31)" in r.stderr


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference sources absent (GPU box)")
def test_reference_cli_builds_against_the_dropin():
    """the reference's main.cpp, unmodified, over include/dropin + libskq.so."""
    subprocess.run(["make", "-s", "-C", ROOT, "-f", "oracle/ref.mk", "all"], check=True)
    for exe in CLIS:
        assert os.access(exe, os.X_OK)
        out = subprocess.run([exe, "-h"], capture_output=True, text=True, check=True).stdout
        assert "quant <index_file> <reads.fastq> <output>" in out
        nm = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
        # the hot path comes from libskq.so: the sketch and the chain are undefined in the binary
        assert "createSketch_FracMinhash_direct" in nm and "sparse_chain" in nm
    nm_all = subprocess.run(["nm", "-D", "--undefined-only", CLIS[1]], capture_output=True, text=True,
                            check=True).stdout
    for sym in ("load_index", "load_fasta", "save_index", "output_to_csv", "estimate_isoform_abundance_em"):
        assert sym in nm_all, sym


def _rows(path):
    lines = open(path).read().splitlines()
    assert lines[0] == "Name,NumReads,EM_Abundance"
    return {tuple(l.split(",")) for l in lines[1:]}


def _run(exe, *args):
    return subprocess.run([exe, *map(str, args)], check=True, capture_output=True, text=True, timeout=600).stdout


need_bins = pytest.mark.skipif(not all(os.access(e, os.X_OK) for e in CLIS),
                               reason="reference CLI not built (oracle/ref.mk needs /root/reference)")


@pytest.mark.gpu
@need_bins
@pytest.mark.parametrize("exe", CLIS, ids=["ref_io", "skq_io"])
def test_reference_cli_edge_fixture(tmp_path, exe):
    idx, csv = tmp_path / "e.idx", tmp_path / "e.csv"
    out = _run(exe, "-k", "31", "-o", "index", os.path.join(EDGE, "e.fa"), idx)
    assert "Index built in" in out and "Index saved to" in out
    out = _run(exe, "-o", "quant", idx, os.path.join(EDGE, "e.fq"), csv)
    assert "Sparse chaining completed" in out and "Output written to" in out
    assert _rows(csv) == {("T2", "2", "2.01333"), ("T4last", "1", "1.01333")}


@pytest.mark.gpu
@need_bins
def test_reference_cli_agrees_with_skq_cli(tmp_path):
    tx = synth.transcriptome(120, seed=71)
    fa, fq = tmp_path / "t.fa", tmp_path / "r.fq"
    tx.write_fasta(fa)
    bases, _, _ = synth.reads(tx, 1500, 150, seed=72)
    rng = random.Random(73)
    with open(fq, "wb") as f:
        for i in range(1500):
            s = bases[i * 150:(i + 1) * 150].tobytes()
            if i % 97 == 0:
                s = s[:60] + b"N" + s[61:]
            f.write(b"@r%d\n%s\n+\n%s\n" % (rng.randrange(1400), s, b"I" * len(s)))  # ids repeat
    ks = "21,31"
    got = {}
    for name, exe in (("ref_io", CLIS[0]), ("skq_io", CLIS[1]), ("skq", SKQ)):
        idx, csv = tmp_path / (name + ".idx"), tmp_path / (name + ".csv")
        _run(exe, "-k", ks, "-o", "index", fa, idx)
        _run(exe, "-o", "quant", idx, fq, csv)
        got[name] = {r[0]: (float(r[1]), float(r[2])) for r in _rows(csv)}
    # each index file read by the other implementations (the reference's save_index / load_index
    # against skq's writer and reader)
    _run(CLIS[0], "-o", "quant", tmp_path / "skq.idx", fq, tmp_path / "x1.csv")
    _run(SKQ, "-o", "quant", tmp_path / "ref_io.idx", fq, tmp_path / "x2.csv")
    got["ref_io<-skq.idx"] = {r[0]: (float(r[1]), float(r[2])) for r in _rows(tmp_path / "x1.csv")}
    got["skq<-ref_io.idx"] = {r[0]: (float(r[1]), float(r[2])) for r in _rows(tmp_path / "x2.csv")}
    base = got["skq"]
    assert len(base) > 60
    for name, g in got.items():
        assert set(g) == set(base), name
        for t, (c, p) in base.items():  # 6 printed digits; EM sums in another order
            assert g[t][0] == pytest.approx(c, rel=5e-6, abs=1e-9), (name, t)
            assert g[t][1] == pytest.approx(p, rel=5e-6), (name, t)


def _timed(exe, *args):
    """(stdout lines with the seconds since start at which each appeared, total seconds)"""
    import time
    t0 = time.perf_counter()
    p = subprocess.Popen([exe, *map(str, args)], stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = []
    for ln in p.stdout:
        lines.append((time.perf_counter() - t0, ln.rstrip()))
    assert p.wait(timeout=600) == 0
    return lines, time.perf_counter() - t0


@pytest.mark.gpu
@need_bins
def test_reference_cli_timing_200tx_100k_reads(tmp_path):
    """The reference's own main.cpp over the drop-in (one GPU call per sequence per k at
    src/main.cpp:79 and :143-144, batched sparse_chain) against the skq CLI, 200 transcripts x
    100k 150-bp reads, k = 31: phase times from the reference's progress lines."""
    tx = synth.transcriptome(200, seed=81)
    fa, fq = tmp_path / "t.fa", tmp_path / "r.fq"
    tx.write_fasta(fa)
    n = 100_000
    bases, _, _ = synth.reads(tx, n, 150, seed=82)
    with open(fq, "wb") as f:
        f.write(synth.fastq_bytes(bases, 150).tobytes())
    rows = {}
    for name, exe in (("ref_cli_skq", CLIS[0]), ("skq", SKQ)):
        idx, csv = tmp_path / (name + ".idx"), tmp_path / (name + ".csv")
        li, ti = _timed(exe, "-k", "31", "-o", "index", fa, idx)
        lq, tq = _timed(exe, "-o", "quant", idx, fq, csv)
        rows[name] = {r[0]: (float(r[1]), float(r[2])) for r in _rows(csv)}
        print("%s: index %.2fs, quant %.2fs; quant progress: %s" % (
            name, ti, tq, "; ".join("%.2fs %s" % (t, l[:40]) for t, l in lq)))
    assert set(rows["ref_cli_skq"]) == set(rows["skq"])
