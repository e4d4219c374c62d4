"""Per-read digests of an skq export — TEST INFRASTRUCTURE, the numpy restatement of
oracle/oracle.c orc_map_digest (its header states the definition): per read, the splitmix64 items of
its status, its retained hashes per k slot (ascending, position j) and its candidates (tid and score
at position j), summed mod 2^64. Equal digests read by read mean equal per-read results."""
import numpy as np

M1 = np.uint64(0xbf58476d1ce4e5b9)
M2 = np.uint64(0x94d049bb133111eb)


def mix64(x):
    x = x ^ (x >> np.uint64(30))
    x = x * M1
    x = x ^ (x >> np.uint64(27))
    x = x * M2
    return x ^ (x >> np.uint64(31))


def item(tag, j, v):
    """tag: scalar or array; j, v: arrays (uint64)."""
    t = np.asarray(tag, np.uint64) << np.uint64(56)
    return mix64(t ^ (np.asarray(j, np.uint64) << np.uint64(32)) ^ np.asarray(v, np.uint64))


def _seg_sums(vals, offs):
    """per segment [offs[i], offs[i+1]) the sum of vals mod 2^64 (empty segments: 0)."""
    cs = np.zeros(len(vals) + 1, np.uint64)
    if len(vals):
        np.cumsum(vals, dtype=np.uint64, out=cs[1:])
    o = np.asarray(offs, np.int64)
    return cs[o[1:]] - cs[o[:-1]]


def export_digest(out, nk):
    """out: skq Session.export() (status, hash_offs, hashes, cand_offs, cand_tid, cand_score)."""
    st = np.asarray(out["status"]).astype(np.uint64)
    n = len(st)
    d = item(0xA5, np.zeros(n, np.uint64), st)
    ho = np.asarray(out["hash_offs"], np.int64)
    nh = int(ho[-1])
    if nh:
        lens = np.diff(ho)
        seg = np.repeat(np.arange(n * nk, dtype=np.int64), lens)
        j = np.arange(nh, dtype=np.int64) - ho[seg]
        slot = (seg % nk) + 1
        del seg
        it = item(slot.astype(np.uint64), j.astype(np.uint64), np.asarray(out["hashes"][:nh], np.uint64))
        del slot, j
        d += _seg_sums(it, ho[::nk])
        del it
    co = np.asarray(out["cand_offs"], np.int64)
    nc = int(co[-1])
    if nc:
        seg = np.repeat(np.arange(n, dtype=np.int64), np.diff(co))
        j = (np.arange(nc, dtype=np.int64) - co[seg]).astype(np.uint64)
        del seg
        it = item(0xC0, j, np.asarray(out["cand_tid"][:nc], np.uint64)) + \
            item(0xD0, j, np.asarray(out["cand_score"][:nc], np.uint64))
        d += _seg_sums(it, co)
    return d
