"""Pin the oracle before trusting it (CPU only).

Ground truth:
  * ntHash's constant tables, read as data from the reference's prebuilt binary
    (tests/golden/nthash_tables.json, made by tests/golden/make_nthash_tables.py);
  * the known-answer vectors recorded in SURVEY.md §8c;
  * the reference source semantics (threshold, set semantics, chain filter).
"""
import json
import math
import os
import random

import numpy as np
import pytest

import orc

HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = {k: [int(v, 16) if isinstance(v, str) else v for v in vals]
          for k, vals in json.load(open(os.path.join(HERE, "golden", "nthash_tables.json")))["tables"].items()}
SEED = TABLES["SEED_TAB"]
CONV = TABLES["CONVERT_TAB"]
M64 = (1 << 64) - 1


def srol(x, d=1):
    for _ in range(d):
        x = ((x << 1) & 0xFFFFFFFDFFFFFFFF) | ((x & 0x8000000000000000) >> 30) | ((x & 0x100000000) >> 32)
    return x


def table_forward_hash(s: bytes, k: int) -> int:
    """ntHash2's base_forward_hash structure: tetramer blocks then the 1-3 base remainder, all
    through the binary's TETRAMER/TRIMER/DIMER/SEED tables indexed via CONVERT_TAB."""
    TET, TRI, DI = TABLES["TETRAMER_TAB"], TABLES["TRIMER_TAB"], TABLES["DIMER_TAB"]
    c = [CONV[b] for b in s[:k]]
    h = 0
    for i in range(0, k - 3, 4):
        h = srol(h, 4) ^ TET[64 * c[i] + 16 * c[i + 1] + 4 * c[i + 2] + c[i + 3]]
    r = k % 4
    i = k - r
    if r == 3:
        h = srol(h, 3) ^ TRI[16 * c[i] + 4 * c[i + 1] + c[i + 2]]
    elif r == 2:
        h = srol(h, 2) ^ DI[4 * c[i] + c[i + 1]]
    elif r == 1:
        h = srol(h, 1) ^ SEED[s[i]]
    return h


def rand_seq(rng, n, alphabet=b"ACGT"):
    return bytes(rng.choice(alphabet) for _ in range(n))


def test_seed_table_matches_oracle():
    lib = orc.lib()
    for c in range(256):
        if CONV[c] != 255:
            assert lib.orc_seed(c) == SEED[c], chr(c)
        else:
            # bytes 0x01,0x03,0x04,0x05,0x07 carry seeds in ntHash's SEED_TAB but no CONVERT_TAB
            # code (ntHash itself is inconsistent on them); the oracle and product treat them as N.
            assert lib.orc_seed(c) == 0
    assert sum(1 for c in range(256) if CONV[c] != 255) == 10  # ACGTU acgtu


@pytest.mark.parametrize("b", "ACGT")
def test_split_rotate_tables(b):
    seed = SEED[ord(b)]
    L, R = TABLES[b + "31L"], TABLES[b + "33R"]
    for i in range(70):
        assert (L[i % 31] | R[i % 33]) == srol(seed, i)
        assert orc.lib().orc_srol(srol(seed, i)) == srol(seed, i + 1)


def test_multimer_tables_compose():
    inv = "ACGT"
    S = [SEED[ord(x)] for x in inv]
    DI, TET = TABLES["DIMER_TAB"], TABLES["TETRAMER_TAB"]
    for a in range(4):
        for b in range(4):
            assert DI[4 * a + b] == srol(S[a]) ^ S[b]
            for c in range(4):
                for d in range(4):
                    assert TET[64 * a + 16 * b + 4 * c + d] == srol(S[a], 3) ^ srol(S[b], 2) ^ srol(S[c]) ^ S[d]


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 19, 21, 25, 31, 32, 33, 34, 63, 64, 65, 100])
def test_rolling_equals_table_hash(k):
    rng = random.Random(k)
    for trial in range(6):
        s = rand_seq(rng, rng.randint(k, k + 120), b"ACGTacgtUu")
        hs, pos = orc.nthash_fwd(s, k)
        assert pos == list(range(len(s) - k + 1))
        assert hs == [table_forward_hash(s[j:j + k], k) for j in range(len(s) - k + 1)]


@pytest.mark.parametrize("k", [3, 5, 21, 31])
def test_invalid_bases_are_skipped(k):
    rng = random.Random(100 + k)
    for trial in range(20):
        s = bytearray(rand_seq(rng, rng.randint(k, 200)))
        for _ in range(rng.randint(0, 4)):
            s[rng.randrange(len(s))] = rng.choice(b"NnX.\x01-")
        s = bytes(s)
        hs, pos = orc.nthash_fwd(s, k)
        expect = [j for j in range(len(s) - k + 1) if all(CONV[c] != 255 for c in s[j:j + k])]
        assert pos == expect
        assert hs == [table_forward_hash(s[j:j + k], k) for j in expect]


def test_argument_errors():
    with pytest.raises(ValueError):
        orc.nthash_fwd(b"ACG", 4)
    with pytest.raises(ValueError):
        orc.nthash_fwd(b"ACG", 0)


def lcg_seq(n, x=42):
    out = []
    for _ in range(n):
        x = (x * 6364136223846793005 + 1442695040888963407) % (1 << 64)
        out.append("ACGT"[x >> 62])
    return "".join(out).encode()


S2 = (b"GACGGAAACACGTCTCTACGCCCCCGGCCGTGCGAGACTGATTTCTCAAAGCAGACCTACCATTCATTCATTATCCAGCTGCGCGGG"
      b"TGGTGATAATCGAATTCGCCCGATGCGGTTCTTTCGAAGATCGGGAGTGATAACAATGTGGAC")


def test_known_answer_vectors_survey_8c():
    assert orc.threshold() == 214748367
    assert int(4294967295 * 0.05) == 214748364  # the double literal would differ: it is NOT used
    hs, _ = orc.nthash_fwd(b"ACGT" * 8, 31)
    assert hs == [0xA11AB471672CE8D2, 0x57EBDAA5E0CA14EE]
    assert [h & 0xFFFFFFFF for h in hs] == [1730996434, 3771340014]
    hs, _ = orc.nthash_fwd(b"A" * 31, 31)
    assert hs == [0xFFFFFFFEAF928327] and hs[0] & 0xFFFFFFFF == 2945614631
    m33 = (1 << 33) - 1
    rot = {"A": [0x08E995C60, 0x0E995C604, 0x06571811D], "C": [0x169962A02, 0x09962A02B, 0x058A80AD3],
           "G": [0x064882572, 0x048825723, 0x02095C8C9], "T": [0x08AD4BE24, 0x0AD4BE244, 0x152F89115]}
    for b, vals in rot.items():
        assert [srol(SEED[ord(b)], k) & m33 for k in (21, 25, 31)] == vals
    assert lcg_seq(150) == S2
    assert orc.sketch(S2, 31) == [6901433, 28017476, 62078630, 110941329, 117651234, 183192842]
    assert orc.sketch(S2, 25) == [88484980, 133066473, 151175954, 184611694, 193294427, 201980600]
    assert orc.sketch(S2, 21) == [29420402, 94748412, 120647760, 139062943, 167579431, 171073265,
                                  181486452, 184699877, 190714733]
    hs, _ = orc.nthash_fwd(S2, 31)
    assert [h & 0xFFFFFFFF for h in hs[:3]] == [2113525738, 1496400953, 3048415779]


def test_sketch_is_threshold_set():
    rng = random.Random(5)
    for k in (21, 31):
        s = rand_seq(rng, 2000)
        hs, _ = orc.nthash_fwd(s, k)
        assert orc.sketch(s, k) == sorted({h & 0xFFFFFFFF for h in hs if h & 0xFFFFFFFF <= 214748367})
        # repeats collapse (set semantics of std::unordered_set)
        rep = s[:300] * 3
        hs, _ = orc.nthash_fwd(rep, k)
        assert orc.sketch(rep, k) == sorted({h & 0xFFFFFFFF for h in hs if h & 0xFFFFFFFF <= 214748367})


def test_chain_filter_equivalence():
    # count >= fl(0.9*m)  <=>  10*count >= 9*m for every m the path can produce
    for m in range(0, 100001):
        assert math.ceil(0.9 * m) == -(-9 * m // 10)


def test_is_valid_sequence():
    lib = orc.lib()
    assert lib.orc_is_valid_sequence(b"ACGTTGCA", 8) == 1
    assert lib.orc_is_valid_sequence(b"", 0) == 1
    for bad in (b"ACGN", b"acgt", b"ACGU", b"ACG\r", b"AC GT"):
        assert lib.orc_is_valid_sequence(bad, len(bad)) == 0


def test_chain_read_semantics_small():
    # Hand-built index: k=31 only. tid0 shares hashes {1,2,3}, tid1 {1,2}, tid2 {9}
    ix = orc.Index([31], pairs=[(np.array([1, 2, 3, 1, 2, 9], np.uint32),
                                 np.array([0, 0, 0, 1, 1, 2], np.uint32))], ntx=3)
    res = ix.map_batch.__func__  # noqa: F841  (batch path covered elsewhere)
    import ctypes as C
    h = np.array([1, 2, 3, 9], np.uint32)
    hp = (C.c_void_p * 1)(h.ctypes.data)
    nh = np.array([4], np.uint32)
    pres = np.array([1], np.int32)
    t = np.zeros(8, np.uint32)
    s = np.zeros(8, np.uint32)
    n = orc.lib().orc_chain_read(ix.h, hp, orc.ptr(nh), orc.ptr(pres), 0.9, orc.ptr(t), orc.ptr(s), 8)
    # counts: t0=3, t1=2, t2=1; max 3, thr 2.7 -> only t0
    assert n == 1 and t[0] == 0 and s[0] == 3
    n = orc.lib().orc_chain_read(ix.h, hp, orc.ptr(nh), orc.ptr(pres), 0.5, orc.ptr(t), orc.ptr(s), 8)
    assert n == 2 and list(t[:2]) == [0, 1] and list(s[:2]) == [3, 2]
    n = orc.lib().orc_chain_read(ix.h, hp, orc.ptr(nh), orc.ptr(pres), 0.0, orc.ptr(t), orc.ptr(s), 8)
    assert n == 3 and list(t[:3]) == [0, 1, 2]
    # absent k: max 0 -> threshold 0 -> everything passes with score 0 contribution
    pres0 = np.array([0], np.int32)
    n = orc.lib().orc_chain_read(ix.h, hp, orc.ptr(nh), orc.ptr(pres0), 0.9, orc.ptr(t), orc.ptr(s), 8)
    assert n == 0
