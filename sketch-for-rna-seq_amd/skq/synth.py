"""Seeded synthetic transcriptome + reads, numpy only.

Transcriptome: genes of 3-10 exons of U[80,400] uniform-ACGT bases; 1-6 isoforms per gene, each
keeps exon 0 and every other exon with p = 0.7 (isoforms share exons, so postings lists hold
several transcripts, as in GENCODE). Headers are GENCODE-style (~75 chars).
Reads: forward strand (the reference hashes forward k-mers only), uniform transcript among
those at least `read_len` long, uniform start, substitutions at rate `err`, quality 'I'.
"""
import numpy as np

ACGT = np.frombuffer(b"ACGT", np.uint8)


class Transcriptome:
    def __init__(self, seqs, offs, names):
        self.seqs = seqs      # uint8, concatenated
        self.offs = offs      # uint64, ntx + 1
        self.names = names    # list of str (FASTA ids: header up to the first space)

    @property
    def ntx(self):
        return len(self.offs) - 1

    def seq(self, t):
        return self.seqs[int(self.offs[t]):int(self.offs[t + 1])].tobytes()

    def write_fasta(self, path, width=60):
        with open(path, "wb") as f:
            for t in range(self.ntx):
                f.write(b">" + self.names[t].encode() + b"\n")
                s = self.seq(t)
                for i in range(0, len(s), width):
                    f.write(s[i:i + width] + b"\n")


def transcriptome(ntx, seed=1):
    rng = np.random.default_rng(seed)
    pieces, lens, names = [], [], []
    g = 0
    while len(lens) < ntx:
        n_ex = int(rng.integers(3, 11))
        ex_len = rng.integers(80, 401, n_ex)
        exons = ACGT[rng.integers(0, 4, int(ex_len.sum()))]
        bounds = np.concatenate([[0], np.cumsum(ex_len)])
        n_iso = int(rng.integers(1, 7))
        for i in range(n_iso):
            if len(lens) >= ntx:
                break
            keep = rng.random(n_ex) < 0.7
            keep[0] = True
            parts = [exons[bounds[j]:bounds[j + 1]] for j in range(n_ex) if keep[j]]
            s = np.concatenate(parts)
            t = len(lens)
            names.append("ENSTSYN%08d.1|ENSGSYN%06d.1|-|-|SYN%d-%03d|SYN%d|%d|protein_coding|"
                         % (t, g, g, i, g, len(s)))
            pieces.append(s)
            lens.append(len(s))
        g += 1
    offs = np.zeros(ntx + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    return Transcriptome(np.concatenate(pieces), offs, names)


def reads(tx, n, read_len, seed=2, err=0.001, chunk=1 << 20):
    """Returns (flat uint8 bases of n * read_len, origin tid per read, start per read)."""
    rng = np.random.default_rng(seed)
    lens = np.diff(tx.offs).astype(np.int64)
    elig = np.nonzero(lens >= read_len)[0]
    if len(elig) == 0:
        raise ValueError("no transcript is long enough")
    out = np.empty(n * read_len, np.uint8)
    tids = elig[rng.integers(0, len(elig), n)]
    starts = (rng.random(n) * (lens[tids] - read_len + 1)).astype(np.int64)
    ar = np.arange(read_len, dtype=np.int64)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        base = tx.offs[tids[a:b]].astype(np.int64) + starts[a:b]
        blk = tx.seqs[(base[:, None] + ar[None, :]).ravel()]
        if err > 0:
            m = rng.random(blk.shape[0]) < err
            blk[m] = ACGT[rng.integers(0, 4, int(m.sum()))]
        out[a * read_len:b * read_len] = blk
    return out, tids, starts


def write_fastq(path, bases, read_len, tids=None, starts=None, names=None):
    n = len(bases) // read_len
    q = b"I" * read_len
    with open(path, "wb") as f:
        for r in range(n):
            hdr = b"@read%d" % r
            if tids is not None:
                tn = names[tids[r]].split("|")[0] if names else str(tids[r])
                hdr += b" tx=%s pos=%d" % (tn.encode(), int(starts[r]))
            f.write(hdr + b"\n" + bases[r * read_len:(r + 1) * read_len].tobytes() + b"\n+\n" + q + b"\n")


def fastq_bytes(bases, read_len, first=0):
    """FASTQ text of fixed-length reads (vectorised): `@read<9-digit ordinal>`, the bases, `+`,
    quality all 'I' — the record layout write_fastq uses, with fixed-width ids."""
    n = len(bases) // read_len
    hdr = 1 + 4 + 9 + 1
    rs = hdr + read_len + 1 + 2 + read_len + 1
    out = np.empty((n, rs), np.uint8)
    out[:, 0:5] = np.frombuffer(b"@read", np.uint8)
    num = np.arange(first, first + n, dtype=np.int64)
    for d in range(9):
        out[:, 5 + 8 - d] = 48 + (num // 10 ** d) % 10
    out[:, hdr - 1] = 10
    out[:, hdr:hdr + read_len] = bases[:n * read_len].reshape(n, read_len)
    o = hdr + read_len
    out[:, o] = 10
    out[:, o + 1] = ord("+")
    out[:, o + 2] = 10
    out[:, o + 3:o + 3 + read_len] = ord("I")
    out[:, rs - 1] = 10
    return out.reshape(-1)
