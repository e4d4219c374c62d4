"""GPU FASTQ ingest (skq_ingest_*): records, statuses, sketches, candidates and the kept-record
rule against a pure-Python restatement of the reference's reader (src/main.cpp:119-147) and the
CPU oracle, bit-exact, across chunk boundaries, halos, sub-batches and malformed input."""
import random

import numpy as np
import pytest

import orc
import skq
from skq import synth


def ref_records(data: bytes):
    """process_fastq_single_pass's loop (src/main.cpp:119-129) as std::getline sees the file:
    [(id, sequence)] for every record, before any filtering."""
    lines = data.split(b"\n")
    if lines[-1] == b"":
        lines.pop()  # a final '\n' ends the last line; an empty file has no lines
    recs, i = [], 0
    while i < len(lines):
        line = lines[i]
        i += 1
        if not line or line[:1] != b"@":
            continue
        seq = lines[i] if i < len(lines) else b""  # getline at EOF leaves an empty string
        i += 3                                      # sequence, '+', quality
        recs.append((line[1:], seq))
    return recs


def ref_kept(recs, ok):
    """read_sketches[read.id] = ... for valid reads only: the last OK record of an id wins."""
    last = {}
    for r, (rid, _) in enumerate(recs):
        if ok[r]:
            last[rid] = r
    kept = np.zeros(len(recs), np.uint8)
    for r in last.values():
        kept[r] = 1
    return kept


def tricky_fastq(tx, n, seed, long_junk=0):
    """FASTQ text with everything the reader's rules care about."""
    rng = random.Random(seed)
    bases, _, _ = synth.reads(tx, n, 150, seed=seed)
    out = []
    ids = []
    for i in range(n):
        seq = bases[i * 150:(i + 1) * 150].tobytes()
        roll = rng.random()
        rid = b"read%d tx=%d" % (i, i % 7)
        if ids and rng.random() < 0.08:       # duplicate id (valid or not)
            rid = rng.choice(ids)
        ids.append(rid)
        qual = b"I" * len(seq)
        nl = b"\n"
        if roll < 0.05:
            qual = b"@" + qual[1:]              # quality line that looks like a header
        elif roll < 0.08:
            seq = seq[:60] + b"N" + seq[61:]
        elif roll < 0.10:
            seq = seq.lower()
        elif roll < 0.12:
            nl = b"\r\n"                         # getline keeps '\r': invalid read
        elif roll < 0.14:
            seq = seq[:rng.randint(0, 30)]       # shorter than k
        elif roll < 0.16:
            seq = seq + seq[:rng.randint(1, 200)]  # longer reads (slow paths past 256 bp)
        elif roll < 0.18:
            out.append(rng.choice([b"junk line", b"", b"+", b"ACGT" * 5]) + b"\n")
        elif roll < 0.19:
            seq = b"@" + seq[1:]                 # sequence line starting with '@': still the sequence
        if long_junk and rng.random() < 0.01:
            out.append(b"x" * long_junk + b"\n")  # lines longer than a chunk
        out.append(b"@" + rid + nl + seq + nl + b"+" + nl + qual + nl)
    return b"".join(out)


def ingest_all(index, path, max_reads, chunk_bytes=0, io_threads=2, fraction=0.9):
    s = skq.Session(index, max_reads, 256)
    g = skq.Ingest(s, path, chunk_bytes=chunk_bytes, io_threads=io_threads)
    status, hashes, cands = [], [], []
    nexp = 0
    while True:
        first, n = g.map(fraction=fraction)
        if n == 0:
            break
        assert first == nexp
        nexp += n
        s.check()
        out = s.export()
        status.append(out["status"].copy())
        ho, co = out["hash_offs"], out["cand_offs"]
        for r in range(n):
            hashes.append(list(out["hashes"][ho[r]:ho[r + 1]]))
            cands.append((list(out["cand_tid"][co[r]:co[r + 1]]), list(out["cand_score"][co[r]:co[r + 1]])))
    kept = g.finish()
    ids = [g.id(r) for r in range(g.records())]
    totals = s.totals()
    g.close()
    st = np.concatenate(status) if status else np.zeros(0, np.uint8)
    return dict(status=st, hashes=hashes, cands=cands, kept=kept, ids=ids, totals=totals)


def test_reader_restatement_matches_host_reader(tmp_path):
    """The Python restatement used as the checker agrees with the host reader (skq_fastq_*)."""
    tx = synth.transcriptome(30, seed=2)
    for seed, junk in ((1, 0), (2, 300)):
        data = tricky_fastq(tx, 400, seed=seed, long_junk=junk) + b"@tail\nAC"
        p = tmp_path / "r.fq"
        p.write_bytes(data)
        q = skq.FastqReader(p)
        first, seqs = q.next(10 ** 6)
        ids = [q.id(r) for r in range(len(seqs))]
        q.close()
        assert list(zip(ids, seqs)) == ref_records(data)


def _machine_states(data):
    """The reader's record-machine state at every line start (src/main.cpp:119-129)."""
    st, s, a = {}, 0, 0
    while a < len(data):
        st[a] = s
        s = (1 if data[a:a + 1] == b"@" else 0) if s == 0 else (s + 1) & 3
        nl = data.find(b"\n", a)
        a = len(data) if nl < 0 else nl + 1
    st[len(data)] = s
    return st


def test_fastq_split_points_and_states(tmp_path):
    """skq_fastq_split: part bounds at line starts, and the exact reader state there, also where
    the four possible states never converge (every line starts with '@': the whole prefix)."""
    tx = synth.transcriptome(30, seed=2)
    cases = [tricky_fastq(tx, 800, seed=3, long_junk=500), b"@x\n" * 20000, b"", b"@a\nAC", b"@a\n" + b"+\n" * 7000]
    for data in cases:
        p = tmp_path / "s.fq"
        p.write_bytes(data)
        st = _machine_states(data)
        for parts in (1, 2, 3, 7):
            offs, states = skq.fastq_split(p, parts)
            assert offs[0] == 0 and offs[-1] == len(data) and all(np.diff(offs.astype(np.int64)) >= 0)
            for q in range(parts):
                o = int(offs[q])
                assert o == 0 or data[o - 1:o] == b"\n"
                assert states[q] == st[o], (q, o)


@pytest.fixture(scope="module")
def tx200():
    tx = synth.transcriptome(200, seed=77)
    seqs = [tx.seq(t) for t in range(tx.ntx)]
    buf, offs = skq.pack_reads(seqs)
    index = skq.Index([31], len(seqs), skq.build_tables(buf, offs, [31]))
    return tx, seqs, index, orc.Index([31], seqs=seqs)


def check_against_reference(res, data, oi):
    recs = ref_records(data)
    assert res["ids"] == [rid for rid, _ in recs]
    n = len(recs)
    assert len(res["status"]) == n
    if n == 0:
        return
    seqs = [s for _, s in recs]
    ref = oi.map_batch(seqs)
    assert np.array_equal(res["status"] & 3, ref["status"])
    for r in range(n):
        c = int(ref["cand_cnt"][r])
        assert res["cands"][r] == (list(ref["cand_tid"][r, :c]), list(ref["cand_score"][r, :c])), r
        assert res["hashes"][r] == list(ref["hashes"][r, 0, :ref["hash_cnt"][r, 0]]), r
    assert np.array_equal(res["kept"], ref_kept(recs, ref["status"] == 0))


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,max_reads", [(0, 100000), (4096, 37), (1 << 16, 1000)])
def test_ingest_matches_reference_reader(tmp_path, tx200, chunk, max_reads):
    tx, _, index, oi = tx200
    data = tricky_fastq(tx, 1500, seed=5)
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    res = ingest_all(index, p, max_reads, chunk_bytes=chunk)
    check_against_reference(res, data, oi)


@pytest.mark.gpu
@pytest.mark.parametrize("parts,chunk", [(2, 0), (3, 4096), (5, 1 << 15)])
def test_ingest_in_parts_matches_reference_reader(tmp_path, tx200, parts, chunk):
    """The file split for several devices (here all on one): every part ingested from its bounds
    and entry state, duplicate ids settled across parts; in file order the records, statuses,
    sketches, candidates and kept flags equal the single reader's."""
    tx, _, index, oi = tx200
    data = tricky_fastq(tx, 1500, seed=5)
    rng = random.Random(parts)
    lines = data.split(b"\n")
    # the same ids again near the end of the file, so duplicates cross the parts
    extra = []
    for _ in range(40):
        i = rng.randrange(0, 1400)
        seq = tx.seq(i % tx.ntx)[:150]
        extra.append(b"@read%d tx=%d\n%s\n+\n%s\n" % (i, i % 7, seq, b"I" * len(seq)))
    data = data + b"".join(extra)
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    offs, states = skq.fastq_split(p, parts)
    res, gs, kepts = [], [], []
    for q in range(parts):
        s = skq.Session(index, 300, 256)
        g = skq.Ingest(s, p, chunk_bytes=chunk, part=(int(offs[q]), int(offs[q + 1]), int(states[q])))
        status, hashes, cands = [], [], []
        while True:
            first, n = g.map(fraction=0.9)
            if n == 0:
                break
            s.check()
            out = s.export()
            status.append(out["status"].copy())
            ho, co = out["hash_offs"], out["cand_offs"]
            for r in range(n):
                hashes.append(list(out["hashes"][ho[r]:ho[r + 1]]))
                cands.append((list(out["cand_tid"][co[r]:co[r + 1]]), list(out["cand_score"][co[r]:co[r + 1]])))
        kepts.append(g.finish())
        gs.append(g)
        res.append((status, hashes, cands, [g.id(r) for r in range(g.records())], s))
    skq.ingest_supersede(gs, kepts)
    merged = dict(status=np.concatenate([np.concatenate(r[0]) if r[0] else np.zeros(0, np.uint8) for r in res]),
                  hashes=sum((r[1] for r in res), []), cands=sum((r[2] for r in res), []),
                  ids=sum((r[3] for r in res), []), kept=np.concatenate(kepts))
    assert len(set(merged["ids"])) < len(merged["ids"])  # duplicate ids present
    check_against_reference(merged, data, oi)
    for g in gs:
        g.close()


@pytest.mark.gpu
def test_ingest_lines_longer_than_a_chunk(tmp_path, tx200):
    tx, _, index, oi = tx200
    data = tricky_fastq(tx, 600, seed=9, long_junk=9000)
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    res = ingest_all(index, p, 64, chunk_bytes=4096)
    check_against_reference(res, data, oi)


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [b"", b"@last", b"@last\n", b"@last\nACGT", b"@last\nACGT\n+\n", b"junk",
                                  b"\n\n\n"])
def test_ingest_file_endings(tmp_path, tx200, tail):
    tx, _, index, oi = tx200
    data = tricky_fastq(tx, 50, seed=11) + tail
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    for chunk in (0, 1024):
        check_against_reference(ingest_all(index, p, 1000, chunk_bytes=chunk), data, oi)


@pytest.mark.gpu
@pytest.mark.parametrize("data", [b"", b"\n", b"no records here\n+\n", b"@", b"@\n\n\n\n@\n"])
def test_ingest_degenerate_files(tmp_path, tx200, data):
    _, _, index, oi = tx200
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    check_against_reference(ingest_all(index, p, 16, chunk_bytes=4096), data, oi)


@pytest.mark.gpu
def test_ingest_duplicate_groups(tmp_path, tx200):
    """Many records per id, valid and not: every group takes the exact host comparison."""
    tx, _, index, oi = tx200
    bases, _, _ = synth.reads(tx, 400, 150, seed=3)
    rng = random.Random(4)
    out = []
    for i in range(400):
        seq = bases[i * 150:(i + 1) * 150].tobytes()
        if rng.random() < 0.3:
            seq = seq.replace(b"A", b"N", 1)
        out.append(b"@dup%d\n%s\n+\n%s\n" % (rng.randrange(40), seq, b"I" * len(seq)))
    data = b"".join(out)
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    check_against_reference(ingest_all(index, p, 128, chunk_bytes=8192), data, oi)


@pytest.mark.gpu
def test_ingest_totals_and_direct_map_agree(tmp_path, tx200):
    """Ingested batches give the same results and totals as skq_map over the same sequences."""
    tx, _, index, _ = tx200
    bases, _, _ = synth.reads(tx, 20000, 150, seed=21)
    seqs = [bases[i * 150:(i + 1) * 150].tobytes() for i in range(20000)]
    data = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, s, b"F" * 150) for i, s in enumerate(seqs))
    p = tmp_path / "r.fq"
    p.write_bytes(data)
    res = ingest_all(index, p, 6000, chunk_bytes=1 << 20, io_threads=4)
    assert res["kept"].sum() == 20000
    s = skq.Session(index, 20000, 150)
    d = skq.DeviceBuffer.from_numpy(np.frombuffer(b"".join(seqs), np.uint8))
    s.map(d.ptr, None, 20000, 150, fixed_len=150)
    s.check()
    out = s.export()
    co = out["cand_offs"]
    for r in range(0, 20000, 7):
        assert res["cands"][r] == (list(out["cand_tid"][co[r]:co[r + 1]]), list(out["cand_score"][co[r]:co[r + 1]]))
    for a, b in zip(res["totals"], s.totals()):
        assert np.array_equal(a, b)
