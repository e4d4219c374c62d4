#!/usr/bin/env python3
"""End-to-end FASTQ throughput of the GPU ingest (skq_ingest_*): file in the page cache ->
records parsed on the device -> sketch + chain -> (optionally) per-read candidates on the host.

usage: tools/ingest_bench.py [--reads N] [--chunk MiB] [--io-threads T] [--export]

Writes a synthetic FASTQ (cfg3 shape: 150 bp reads of the 200k-transcript synthetic
transcriptome, headers like '@read000000001 tx=...') to --path, reads it once to warm the page
cache, then times skq_ingest_map over the whole file. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import torch  # noqa: E402,F401  (one HIP runtime per process, as in bench.py)
import skq  # noqa: E402
from skq import synth  # noqa: E402


def write_fastq(path, bases, n, L, block=1_000_000):
    """Fixed-layout records: '@read%09d tx=synthetic\\n' + seq + '\\n+\\n' + qual + '\\n'."""
    head = len(b"@read%09d tx=synthetic\n" % 0)
    rec = head + L + 1 + 2 + L + 1
    with open(path, "wb") as f:
        for a in range(0, n, block):
            m = min(block, n - a)
            buf = np.empty((m, rec), np.uint8)
            ids = np.char.encode(np.char.mod("@read%09d tx=synthetic\n", np.arange(a, a + m)), "ascii")
            buf[:, :head] = np.frombuffer(b"".join(ids), np.uint8).reshape(m, head)
            buf[:, head:head + L] = bases[a * L:(a + m) * L].reshape(m, L)
            buf[:, head + L:head + L + 3] = np.frombuffer(b"\n+\n", np.uint8)
            buf[:, head + L + 3:head + 2 * L + 3] = ord("I")
            buf[:, -1] = ord("\n")
            f.write(buf.tobytes())
    return n * rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--ntx", type=int, default=200_000)
    ap.add_argument("--chunk", type=int, default=64, help="MiB per chunk")
    ap.add_argument("--io-threads", type=int, default=8)
    ap.add_argument("--batch", type=int, default=2_000_000, help="session max_reads")
    ap.add_argument("--export", action="store_true", help="copy every batch's candidates to the host")
    ap.add_argument("--em", action="store_true",
                    help="quant end to end: candidates appended on the device, EM (20 rounds) + assignment")
    ap.add_argument("--path", default="/tmp/skq_ingest_bench.fq")
    ap.add_argument("--passes", type=int, default=1, help="timed passes (the median is reported)")
    args = ap.parse_args()

    t0 = time.time()
    tx = synth.transcriptome(args.ntx, seed=1)
    tables = skq.build_tables(tx.seqs, tx.offs, [31], nthreads=16)
    index = skq.Index([31], tx.ntx, tables, device=0)
    bases, _, _ = synth.reads(tx, args.reads, 150, seed=1000, err=0.001)
    size = write_fastq(args.path, bases, args.reads, 150)
    with open(args.path, "rb") as f:  # page cache
        while f.read(1 << 28):
            pass
    sess = skq.Session(index, args.batch, 256)
    print("[ingest] setup %.1fs, %.2f GB FASTQ" % (time.time() - t0, size / 1e9), file=sys.stderr, flush=True)

    def run():
        t_a = time.perf_counter()
        g = skq.Ingest(sess, args.path, chunk_bytes=args.chunk << 20, io_threads=args.io_threads)
        em = skq.EMSet(tx.ntx) if args.em else None
        timing["open_s"] = time.perf_counter() - t_a
        tot = 0
        ncand = 0
        while True:
            _, n = g.map(accumulate=True)
            if n == 0:
                break
            tot += n
            if args.export:
                ncand += len(sess.export()["cand_tid"])
            if em is not None:
                em.add_session(sess)
        sess.check()
        t_b = time.perf_counter()
        timing["loop_s"] = t_b - t_a - timing["open_s"]
        kept = g.finish()
        g.close()
        timing["finish_close_s"] = time.perf_counter() - t_b
        if em is not None:
            t1 = time.perf_counter()
            em.select(kept)
            pi, it = em.run(20, 0.01)
            counts, assigned = em.assign()
            timing["em_s"] = time.perf_counter() - t1
            timing["em_rounds"] = it
            timing["assigned_tx"] = int(assigned.sum())
            em.free()
        return tot, int(kept.sum()), ncand

    timing = {}
    run()  # warm-up (allocations, code objects)
    dts = []
    for _ in range(args.passes):
        sess.reset_totals()
        ts = time.perf_counter()
        n, kept, ncand = run()
        dts.append(time.perf_counter() - ts)
    dt = sorted(dts)[len(dts) // 2]
    res = {"what": "GPU FASTQ ingest end to end (page cache -> parsed on device -> sketch + chain%s)"
                   % (" -> candidates on host" if args.export else ""),
           "reads": n, "kept": kept, "seconds_median": dt, "reads_per_s": n / dt, "fastq_GB_per_s": size / dt / 1e9,
           "pass_reads_per_s": [round(n / d / 1e6, 1) for d in dts], "chunk_MiB": args.chunk, "io_threads": args.io_threads, "batch": args.batch,
           "candidates_exported": ncand if args.export else None}
    if args.em:
        res["what"] = "quant end to end on the GPU (page cache -> parse -> sketch + chain -> EM + assignment)"
        res.update(timing)
    print(json.dumps(res), flush=True)
    os.unlink(args.path)


if __name__ == "__main__":
    main()
