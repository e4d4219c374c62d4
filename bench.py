#!/usr/bin/env python3
"""bench.py — reads/s of the quant hot path (FracMinHash sketch + sparse chain) on MI355X.

Workloads (BASELINE.json configs):
  N = 1: cfg3 (the metric's config) — synthetic 10M x 150 bp reads vs a ~200k-transcript
         GENCODE-scale synthetic index, k = 31, sketch fraction (double)0.05f, chain 0.9;
  N > 1: cfg4 — 12.5M x 150 bp reads per GPU, so N = 8 processes the 100M reads of cfg4 per
         step (weak scaling: reads per GPU fixed; N = 2 / 4 process 25M / 50M).
One step = one pass of the hot path over one batch already resident in HBM (skq_map: the fused
sketch + probe + count kernel, the slow paths and the per-transcript totals) plus, for N > 1, the
one RCCL all-reduce of the per-transcript totals (reads, score) over xGMI.

One process per GPU. `python bench.py --gpus N` with N > 1 and no torch.distributed environment
starts its own N ranks (a child `python -m torch.distributed.run`, never an exec) and exits with
their status; the driver may also launch it under torch.distributed.run itself. Reads are
sharded (each rank its own seeded batch), the index is replicated; rank 0 prints one JSON line.

After the timed steps (rank 0): the parity sample — the first --cpu-reads reads of the batch as
FASTQ text through the CPU oracle (oracle/oracle.c, the checker), compared bit-exact with the GPU's
statuses, retained-hash sets, candidate lists and per-transcript totals for the same reads; a
mismatch exits non-zero. At every N the same oracle runs are the CPU baseline (rank 0, its
per-GPU share of the host cores and 1 thread),
and `end_to_end` reports quant as the CLI runs it (FASTQ file -> device parse -> sketch + chain ->
EM + assignment) over the same batch, checked against the in-HBM map's totals; never `value`.
"""
import argparse
import os
import socket
import subprocess
import sys


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=["cfg2", "cfg3", "cfg4", "cfg5"],
                    help="default: cfg3 at N = 1, cfg4 at N > 1")
    ap.add_argument("--reads", type=int, default=0, help="reads per GPU (default: the config's)")
    ap.add_argument("--cpu-reads", type=int, default=2_000_000,
                    help="parity sample / CPU-baseline sample (reads, rank 0)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: the per-GPU share of the affinity set, affinity CPUs "
                         "/ GPUs on the node, capped at OMP_NUM_THREADS when the box sets it)")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the 1-thread CPU timing")
    ap.add_argument("--io-threads", type=int, default=16, help="end to end: FASTQ pread threads per GPU")
    ap.add_argument("--chunk-mb", type=int, default=64, help="end to end: FASTQ chunk (MiB)")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the FASTQ-file -> EM leg reported beside the kernel path")
    ap.add_argument("--preheat", default="none", choices=["none", "matmul", "map1m"],
                    help="development A/B: GPU work before the warmup steps (what the step time's ramp is)")
    ap.add_argument("--no-settle", action="store_true",
                    help="no settling phase before the warmup steps (the memory clocks' ramp then falls in the timed steps)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="development A/B: no per-kernel HIP events in the timed steps (the roofline then has no launch time)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="N = 1, default config: skip the cfg2 and cfg5 legs reported under `configs`")
    ap.add_argument("--dist-backend", default="nccl",
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on one GPU)")
    return ap.parse_args(argv)


def _spawn_ranks(args):
    """--gpus N > 1 outside torch.distributed: N fresh rank processes (nothing here has touched
    the GPU yet), rendezvous on 127.0.0.1; exit with their status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    _a = _args()
    if _a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(_a))

import ctypes as C  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: libskq.so then binds to torch's HIP runtime)
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import skq  # noqa: E402
from skq import dist as sdist  # noqa: E402
from skq import synth  # noqa: E402

METRIC = "reads/sec (quant, 150 bp, k=31) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GATHER_CEIL_GPS = 48.1  # random 32-B gathers per ns from an 8 GiB table (profiles/r1_gather_bench.log)
VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions/s (MI355X_MICROARCH.md: SIMD-32, 2 cycles each)

CONFIGS = {
    "cfg2": dict(ntx=10_000, reads=1_000_000, read_len=100, ks=[31],
                 desc="synthetic 1M x 100 bp reads vs 10k-transcript index, k=31"),
    "cfg3": dict(ntx=200_000, reads=10_000_000, read_len=150, ks=[31],
                 desc="synthetic 10M x 150 bp reads/GPU vs ~200k-transcript index, k=31"),
    "cfg4": dict(ntx=200_000, reads=12_500_000, read_len=150, ks=[31],
                 desc="synthetic 12.5M x 150 bp reads/GPU (100M at 8 GPUs) vs ~200k-transcript index, k=31"),
    "cfg5": dict(ntx=200_000, reads=10_000_000, read_len=150, ks=[21, 25, 31],
                 desc="synthetic 10M x 150 bp reads/GPU vs ~200k-transcript index, k={21,25,31}"),
}


def log(*a):
    print("[bench r%s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def per_read_stats(out, tables, ks, n):
    """h (retained hashes, summed over k), P (postings touched), C (candidates) per read, from
    an export (deterministic given the inputs)."""
    nk = len(ks)
    ho = out["hash_offs"].astype(np.int64)
    hs = out["hashes"]
    P = 0
    for i, k in enumerate(ks):
        keys, offs, _ = tables[k]
        starts = ho[i:-1:nk]
        ends = ho[i + 1::nk]
        lens = ends - starts
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        x = hs[idx]
        pos = np.searchsorted(keys, x)
        pos = np.minimum(pos, len(keys) - 1)
        hit = keys[pos] == x
        P += int((offs[pos + 1].astype(np.int64) - offs[pos].astype(np.int64))[hit].sum())
    return dict(h=len(hs) / n, P=P / n, C=len(out["cand_tid"]) / n)


def parity_check(gpu, gtot, cpu, nk):
    """The GPU export of the sample against the oracle's FASTQ-path outputs, bit-exact: status,
    retained-hash sets per (read, k), candidate lists (tid, score in the normalised order) and the
    per-transcript totals. Returns a list of mismatch descriptions (empty = bit-exact)."""
    bad = []
    n = cpu["n"]
    if len(gpu["status"]) != n:
        return ["read count %d vs %d" % (len(gpu["status"]), n)]
    st = gpu["status"].astype(np.uint8)
    if not np.array_equal(st, cpu["status"]):
        bad.append("status: %d reads differ" % int((st != cpu["status"]).sum()))
    # hashes: CSR (read-major, k-minor) vs dense [n, nk, hcap]
    ho = gpu["hash_offs"].astype(np.int64)
    cnt = np.diff(ho).reshape(n, nk)
    if not np.array_equal(cnt, cpu["hash_cnt"].astype(np.int64)):
        bad.append("retained-hash counts: %d (read, k) differ" % int((cnt != cpu["hash_cnt"]).sum()))
    else:
        hcap = cpu["hashes"].shape[2]
        mask = np.arange(hcap)[None, None, :] < cpu["hash_cnt"][:, :, None]
        if not np.array_equal(cpu["hashes"][mask], gpu["hashes"][:ho[-1]]):
            bad.append("retained hashes differ")
    co = gpu["cand_offs"].astype(np.int64)
    cc = np.diff(co)
    if not np.array_equal(cc, cpu["cand_cnt"].astype(np.int64)):
        bad.append("candidate counts: %d reads differ" % int((cc != cpu["cand_cnt"]).sum()))
    else:
        ccap = cpu["cand_tid"].shape[1]
        mask = np.arange(ccap)[None, :] < cpu["cand_cnt"][:, None]
        if not np.array_equal(cpu["cand_tid"][mask], gpu["cand_tid"][:co[-1]]):
            bad.append("candidate transcripts differ")
        if not np.array_equal(cpu["cand_score"][mask], gpu["cand_score"][:co[-1]]):
            bad.append("candidate scores differ")
    if not (np.array_equal(gtot[0], cpu["tx_reads"]) and np.array_equal(gtot[1], cpu["tx_score"])):
        bad.append("per-transcript totals differ")
    return bad


def end_to_end(index, ntx, bases, d_ptr, n, L, sess, sp, rank=0, world=1, dev=None, batch=2_000_000, io_cfg=(8, 64)):
    """quant as the CLI runs it, beside the kernel-path metric (never `value`): the job's reads as
    ONE FASTQ file in memory (/dev/shm when there is room, else the page cache; each rank writes
    its shard's records at its own offset) -> split at line starts into one part per rank
    (skq_fastq_split) -> each rank pulls its part into pinned buffers, parses the records on its
    device, sketch + chain, candidates appended on the device -> EM (<= 20 rounds) + assignment:
    on one GPU skq_em_run; on N GPUs every round's posterior sums all-reduced over RCCL
    (skq/dist.py em_gpu / assign_gpu, src/main.cpp:165-197). One warm-up pass, then three timed
    passes (median reported; the slowest rank's time each). Check: the per-transcript totals of
    the ingest path, summed over ranks, equal those of the in-HBM map of the same reads, and every
    read is kept."""
    import tempfile
    rs = 2 * L + 19                       # one record of synth.fastq_bytes (fixed-width ids)
    need = world * n * rs
    tmpdir = None
    if rank == 0:
        try:  # a RAM-backed file when there is room (the timed pass reads it from memory either way)
            st = os.statvfs("/dev/shm")
            if st.f_bavail * st.f_frsize > 3 * need:
                tmpdir = "/dev/shm"
        except OSError:
            pass
        fd, path = tempfile.mkstemp(suffix=".fq", dir=tmpdir)
        os.ftruncate(fd, need)
        os.close(fd)
    else:
        path = None
    if world > 1:
        box = [path, tmpdir]
        dist.broadcast_object_list(box, src=0)
        path, tmpdir = box
    try:
        fd = os.open(path, os.O_WRONLY)
        try:
            for a in range(0, n, 1_000_000):  # this rank's records, ids numbered across the job
                m = min(1_000_000, n - a)
                buf = synth.fastq_bytes(bases[a * L:(a + m) * L], L, first=rank * n + a)
                os.pwrite(fd, buf.tobytes(), (rank * n + a) * rs)
        finally:
            os.close(fd)
        if world > 1:
            dist.barrier()
        offs, states = skq.fastq_split(path, world)
        part = (int(offs[rank]), int(offs[rank + 1]), int(states[rank]))
        with open(path, "rb") as f:  # this rank's part into the page cache
            f.seek(part[0])
            left = part[1] - part[0]
            while left > 0:
                got = len(f.read(min(left, 1 << 28)))
                if not got:
                    break
                left -= got
        es = skq.Session(index, batch, 256)
        emr = {}

        def run():
            g = skq.Ingest(es, path, chunk_bytes=io_cfg[1] << 20, io_threads=io_cfg[0], part=part)
            em = skq.EMSet(ntx, device=dev.index if dev is not None else 0)
            tot = 0
            while True:
                _, got = g.map(accumulate=True)
                if got == 0:
                    break
                tot += got
                em.add_session(es)
            es.check()
            kept = g.finish()
            g.close()
            t1 = time.perf_counter()
            em.select(kept)
            if world == 1:
                _, it = em.run(20, 0.01)
                _, assigned = em.assign()
                na = int(assigned.sum())
            else:
                pi, it = sdist.em_gpu(em, 20, 0.01, device=dev)
                _, assigned = sdist.assign_gpu(em, pi)
                na = int(assigned.sum().item())
            emr.update(em_ms=(time.perf_counter() - t1) * 1e3, em_rounds=it, assigned_transcripts=na)
            em.free()
            return tot, int(kept.sum())

        run()
        times = []
        for _ in range(3):  # three timed passes; the median is reported (boxes' host paths vary)
            es.reset_totals()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ts = time.perf_counter()
            got, kept = run()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            times.append(sdist.max_over_ranks(time.perf_counter() - ts, device=dev))
        dt = sorted(times)[1]
        etot = torch.from_numpy(np.stack(es.totals()).astype(np.int64)).to(dev)
        es.free()
        sess.reset_totals(sp)
        sess.map(d_ptr, None, n, L, fixed_len=L, stream=sp, accumulate=True)
        sess.check(sp)
        dtot = torch.from_numpy(np.stack(sess.totals()).astype(np.int64)).to(dev)
        cnt = torch.tensor([got, kept], dtype=torch.int64, device=dev)
        for t in (etot, dtot, cnt):
            sdist.allreduce_totals(t)
        got_all, kept_all = (int(x) for x in cnt.tolist())
        ok = got_all == world * n and kept_all == world * n and torch.equal(etot, dtot)
        return dict(what="quant end to end on %d GPU%s: one FASTQ file (in memory: /dev/shm or the page cache) split "
                         "into one part per GPU -> device parse -> sketch + chain -> EM + assignment%s (the CLI's path; "
                         "not the metric)" % (world, "s" if world > 1 else "",
                                              " with RCCL all-reduces" if world > 1 else ""),
                    reads=got_all, fastq_GB=need / 1e9,
                    fastq_in="/dev/shm" if tmpdir else "page cache (%s)" % os.path.dirname(path), seconds=dt,
                    io_threads=io_cfg[0], chunk_mb=io_cfg[1],
                    reads_per_s=got_all / dt, pass_reads_per_s=[got_all / t for t in times],
                    check="totals equal the in-HBM map's, all reads kept" if ok else "MISMATCH", **emr)
    finally:
        if world > 1:
            dist.barrier()
        if rank == 0:
            os.unlink(path)


def node_gpus(world):
    """GPUs on this node: the KFD topology's GPU nodes (every GPU of the machine, visible or not),
    at least the ranks of this job."""
    n = 0
    try:
        top = "/sys/class/kfd/kfd/topology/nodes"
        for d in os.listdir(top):
            try:
                props = open(os.path.join(top, d, "properties")).read().split("\n")
            except OSError:
                continue
            for ln in props:
                f = ln.split()
                if len(f) == 2 and f[0] == "simd_count" and int(f[1]) > 0:
                    n += 1
    except OSError:
        pass
    return max(n, world, 1)


def cpu_share(args, world):
    """(threads, how they were derived): the per-GPU share of the affinity set, capped at the
    box's CPU share (OMP_NUM_THREADS, which the GPU pool sets per one-GPU box)."""
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    g = node_gpus(world)
    share = max(1, ncpu // g)
    how = "affinity set %d CPUs / %d GPUs on the node = %d" % (ncpu, g, share)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if args.cpu_threads:
        return args.cpu_threads, ncpu, "--cpu-threads %d (%s)" % (args.cpu_threads, how)
    if omp and omp < share:
        return omp, ncpu, how + ", capped at OMP_NUM_THREADS = %d (this box's CPU share)" % omp
    return share, ncpu, how


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_profile_json(name):
    f = os.path.join(ROOT, "profiles", name)
    return (json.load(open(f)), "profiles/" + name) if os.path.exists(f) else (None, None)


def measure(cname, cfg, args, rank, world, dev, gpu, sample, totals_dev=True):
    """One config's leg on this rank's shard: setup (replicated index, seeded reads resident in HBM),
    W untimed + K timed steps bracketed by a barrier and a device sync, then the sample (the first
    `sample` reads mapped alone and exported) and the roofline figures. Returns (line fields,
    context for the checks)."""
    L, ks, n = cfg["read_len"], cfg["ks"], cfg["reads"]
    t0 = time.time()
    tx = synth.transcriptome(cfg["ntx"], seed=1)  # identical on every rank: replicated index
    tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
    # (the transcripts' sequences too: they let the index add the chained tables, SKQ_CHAIN)
    index = skq.Index(ks, tx.ntx, tables, device=gpu, seqs=(tx.seqs, tx.offs))
    bases, _, _ = synth.reads(tx, n, L, seed=1000 + rank, err=0.001)  # rank's shard
    d_reads = torch.from_numpy(bases).to(dev)
    sess = skq.Session(index, n, L)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    totals = torch.zeros(2, tx.ntx, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    log("%s setup %.1fs: %d transcripts, %d reads x %d bp, index %s" % (
        cname, time.time() - t0, tx.ntx, n, L, index.stats()))

    # the collective's own stream: the step's totals are snapshotted on the session's tail stream
    # and all-reduced there, so the next map on the launch stream does not wait for the tail or
    # the all-reduce (the last step's all-reduce is inside the timed region: its synchronize)
    comm = torch.cuda.Stream(dev) if world > 1 else None
    cp_ = C.c_void_p(comm.cuda_stream) if comm is not None else None

    def step():
        sess.map(d_reads.data_ptr(), None, n, L, fixed_len=L, stream=sp)
        if world > 1:  # the one collective: per-transcript totals, summed over ranks (RCCL)
            with torch.cuda.stream(comm):
                sess.totals_async(totals[0].data_ptr(), totals[1].data_ptr(), stream=cp_)
                sdist.allreduce_totals(totals)

    if args.preheat == "matmul":  # ~100 ms of unrelated GPU work (clocks)
        x = torch.randn(8192, 8192, device=dev)
        for _ in range(40):
            x = (x @ x).clamp_(-1, 1)
        torch.cuda.synchronize(dev)
        del x
    elif args.preheat == "map1m":  # the map over the first 1M reads, 60 times (tables, caches)
        for _ in range(60):
            sess.map(d_reads.data_ptr(), None, min(n, 1_000_000), L, fixed_len=L, stream=sp)
        torch.cuda.synchronize(dev)
    # settling (untimed, before the W warmup steps): the step time falls ~20 % over the first ~25
    # memory-heavy batches of a process as the memory clocks ramp (unrelated compute-bound work does
    # not shorten it; profiles/r5_step_curve.log), so the map runs in groups of 5 batches until a
    # group's time is within 1.5 % of the previous one (at most 60 batches)
    settle = 0
    if not args.no_settle:
        prev = None
        for _ in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(5):
                step()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            settle += 5
            g = e0.elapsed_time(e1)
            # (ranks with a collective in their step run the same count: all 30)
            if world == 1 and prev is not None and abs(g - prev) <= 0.015 * prev:
                break
            if world > 1 and settle >= 30:
                break
            prev = g
    for _ in range(args.warmup):
        step()
    sess.check(sp)
    for kind in range(4):
        sess.kernel_time(kind)
    sess.enable_timing(not args.no_kernel_timing)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ts = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    sess.enable_timing(False)
    sess.check(sp)
    # (total ms, launches): sketch / fused map, probe, count, totals (k_bin_sum + fold)
    kt = [sess.kernel_time(kind) for kind in range(4)]
    elapsed = sdist.max_over_ranks(elapsed, device=dev)  # the slowest rank's time
    slow = sess.slow_counts()

    # the sample: the first m reads of this rank's batch, mapped alone (fresh totals), exported
    m = min(n, sample)
    sess.reset_totals(sp)
    sess.map(d_reads.data_ptr(), None, m, L, fixed_len=L, stream=sp, accumulate=True)
    sess.check(sp)
    gout = sess.export()
    gtot = sess.totals()
    st = per_read_stats(gout, tables, ks, m)
    h, P, Cn = st["h"], st["P"], st["C"]
    nk = len(ks)
    # algorithmic bytes per read, per kernel (DESIGN.md "Roofline"); an index lookup is priced at
    # the 8 B (key, list offset) it needs, a posting at its 4 B tid
    fused = kt[1][1] == 0  # no k_probe launches: the sketch kernel probed (direct/rank table)
    # the fused map (k_map1, or its passes for several k: sketch + entry gathers + count), timed as kind 0
    # with no separate count launches
    map1 = kt[2][1] == 0 and kt[0][1] > 0
    count_name = "k_count3" if tx.ntx <= (1 << 22) else "k_count"
    b_chain = 4 * P + 4 + 8 * Cn + 4 * Cn  # postings in, candidates + count + binned totals out
    b_kern = {
        "k_sketch": L + 4 * h + 4 * nk + 1 + ((8 * h + 4 * h + 1) if fused else 0),
        "k_probe": 1 + 4 * nk + 4 * h + 8 * h + 4 * h + 1,
        count_name: 2 + 4 * nk + 4 * h + 4 * P + 4 + 8 * Cn + 4 * Cn,
        "totals": 4 * Cn + 16.0 * tx.ntx / n,
    }
    # (2..4 k slots: one k_map1 pass per k slot, the last merging, timed together as one map)
    fused_name = "k_map1" if nk == 1 else "k_map1 x%d passes" % nk
    if map1:  # the fused kernel: read in, one lookup per hash, postings, hashes + candidates out
        # (one k slot: the candidates leave packed, tid | score << 22 in one word; include/skq.h)
        b_chain_m = b_chain - (4 * Cn if nk == 1 else 0)
        b_kern = {fused_name: L + 1 + 4 * nk + 4 * h + 8 * h + b_chain_m, "totals": b_kern["totals"]}
    b_path = L + 8 * h + 4 * P + 4 * h + 8 * Cn         # SURVEY.md §8d formula
    names = (fused_name if map1 else "k_sketch", "k_probe", count_name, "totals")
    avg = {name: ms / cnt for name, (ms, cnt) in zip(names, kt) if cnt}
    if not avg:  # (--no-kernel-timing: the step time stands in for the map's launch time)
        avg = {names[0]: elapsed * 1e3 / args.steps}
    # the roofline's kernel: the fused map where it ran (the hot path: sketch + lookups + chain in
    # one launch; the totals kernels beside it on the side stream are not the path's bound, and
    # their HIP-event times stretch with the overlap), else the longest launch
    kname = names[0] if map1 and names[0] in avg else max(avg, key=avg.get)
    # roofline basis: SURVEY.md §8(d)'s algorithmic bytes per read (b_path) when the dominant launch
    # is the fused map (the whole hot path: sketch + lookups + chain in it); the kernel's own
    # input/output bytes (b_kern: + the status byte, hash counts, the binned totals) reported beside
    b_basis = b_path if kname == fused_name else b_kern[kname]
    achieved = n * b_basis / (avg[kname] * 1e-3) / 1e9
    kio = n * b_kern[kname] / (avg[kname] * 1e-3) / 1e9
    traffic, traffic_src = None, None
    # (cfg4 is cfg3's reads, index and k at 12.5M reads per GPU: its per-read traffic is cfg3's)
    tname = "cfg3" if cname == "cfg4" and not os.path.exists(os.path.join(ROOT, "profiles", "traffic_cfg4.json")) else cname
    probe = index.stats()["probe"]
    chained = index.stats()["chained"] > 0
    tr, tf = load_profile_json("traffic_%s.json" % tname)
    if tr is not None:                                   # PMC FETCH/WRITE passes (tools/traffic.py)
        if kname in tr.get("kernels", {}) and tr.get("probe", probe) == probe and "calibration" in tr:
            traffic = tr["kernels"][kname]["hbm_bytes_per_read"] * n
            traffic_src = "%s (%s)%s; %s" % (
                tf, tr.get("measured", "builder's PMC passes"),
                ", per read, scaled to this launch's reads (cfg4 = cfg3's reads, index and k)" if tname != cname else "",
                tr["calibration"])
    # the second bound (K1 "may be ALU- rather than HBM-bound; report both"): the
    # dominant kernel's vector instructions per read from committed PMC passes (SQ_INSTS_VALU over
    # SQ_WAVES x 64 reads, tools/valu_counts.py) over this line's own launch time, against the
    # chip's VALU issue peak
    valu = None
    vj, vf = load_profile_json("valu_%s.json" % tname)
    if vj is not None and kname in vj.get("kernels", {}) and vj.get("probe", probe) == probe \
            and vj.get("chained", chained) == chained:
        vk = vj["kernels"][kname]
        per_launch = vk["valu_per_read"] * n
        va = per_launch / (avg[kname] * 1e-3)
        valu = {"instructions_per_read": vk["valu_per_read"], "per_wave": vk["valu_per_read"] * 64,
                "per_launch": per_launch, "achieved": va, "peak": VALU_PEAK, "unit": "wave64 VALU instructions/s",
                "issue_frac": va / VALU_PEAK, "salu_per_read": vk.get("salu_per_read"),
                "issue_note": ("an issue-COUNT fraction: instructions over the full-rate issue peak (2 cycles per "
                               "wave64 instruction); three-operand forms issue at about half that rate "
                               "(profiles/r4_valu_rate.log), and the counters give no VALU-busy cycles on this "
                               "stack (SQ_ACTIVE_INST_VALU equals the instruction count; DESIGN.md section 5)"),
                "source": "%s (%s)" % (vf, vj.get("measured", "builder's PMC passes")),
                "peak_source": "MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, a wave64 VALU instruction issues over 2 "
                               "cycles, 2.4 GHz -> 1.229e12 wave-instructions/s"}
    hbm_frac = achieved / HBM_PEAK_GBS
    requests = None
    if map1 and traffic is not None:  # every memory-side request of the launch, from the calibrated PMC passes
        kt_ = tr["kernels"][kname]
        per = kt_["fetch_size_bytes_per_read"] / 64.0 + kt_["write_bytes_per_read"] / 64.0
        ra = n * per / (avg[kname] * 1e-3) / 1e9
        requests = {"per_read": per, "achieved": ra, "ceiling": GATHER_CEIL_GPS, "unit": "G requests/s",
                    "frac": ra / GATHER_CEIL_GPS, "hashes_per_read": h,
                    "note": "memory-side read + write requests per read from %s (FETCH_SIZE and WRITE_SIZE "
                            "tally 64 B per request) over the launch time, against the measured random-gather "
                            "ceiling (tools/micro/gather_bench: 46-49 G/s from HBM, 54-56 G/s from the Infinity "
                            "Cache; DESIGN.md section 5)" % tf}
    # the bound: the resource nearest its ceiling, or "latency" when none is above 0.7 (then the
    # kernel waits on dependencies and instruction issue of ~4.5 resident waves per SIMD: the counter
    # file named in bound_evidence)
    fr = {"hbm": hbm_frac}
    if valu is not None:
        fr["valu_issue"] = valu["issue_frac"]
    if requests is not None:
        fr["requests"] = requests["frac"]
    top = max(fr, key=fr.get)
    bound = top if fr[top] >= 0.7 else "latency"
    bj, bf = load_profile_json("pmc_bound_%s.json" % tname)
    bound_ev = None
    if bj is not None and bj.get("kernel") == kname:
        bound_ev = dict(bj.get("derived", {}), source=bf, measured=bj.get("measured"))
    value = n * world * args.steps / elapsed
    line = {
        "value": value, "ms_per_step": elapsed / args.steps * 1e3,
        "settle_steps": settle,
        "roofline": {"bound": bound, "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": hbm_frac, "traffic": traffic,
                     "bound_note": ("achieved / peak / frac are the HBM roofline on SURVEY.md 8(d)'s algorithmic "
                                    "bytes; valu (issue count) and requests (memory-side requests) are the same "
                                    "launch against their ceilings; bound names the largest fraction, or latency "
                                    "when none reaches 0.7"),
                     "fractions": fr, "bound_evidence": bound_ev,
                     "algorithmic_bytes": n * b_basis, "avg_launch_ms": avg[kname],
                     "bytes_basis": ("SURVEY.md 8(d): L + 8h + 4P + 4h + 8C per read" if b_basis == b_path
                                     else "kernel input/output bytes"),
                     "kernel_io_bytes": n * b_kern[kname], "kernel_io_frac": kio / HBM_PEAK_GBS,
                     "valu": valu, "requests": requests,
                     "traffic_GBps": traffic / (avg[kname] * 1e-3) / 1e9 if traffic else None,
                     "traffic_source": traffic_src},
        "path": {"bytes_per_read": b_path, "probe": (fused_name + " (sketch + index gathers + count fused)" if map1 else
                                            "fused in k_sketch" if fused else "k_probe"),
                 "index": index.stats(), "achieved_GBps": value / world * b_path / 1e9,
                 "frac": value / world * b_path / 1e9 / HBM_PEAK_GBS,
                 "kernel_ms": avg, "kernel_bytes_per_read": b_kern, "h": h, "P": P, "C": Cn,
                 "slow_reads_per_batch": {"sketch": slow[0], "chain": slow[1],
                                          "past_the_wave_path": {"sketch": slow[2], "chain": slow[3]}}},
    }
    ctx = dict(tx=tx, tables=tables, index=index, bases=bases, d_reads=d_reads, sess=sess, sp=sp, gout=gout,
               gtot=gtot, m=m, L=L, ks=ks, n=n)
    return line, ctx


def oracle_index(ctx):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc  # the CPU oracle: the checker and the CPU baseline, never the measured path
    pairs = []
    for k in ctx["ks"]:
        keys, offs, tids = ctx["tables"][k]
        pairs.append((np.repeat(keys, np.diff(offs.astype(np.int64))), tids))
    return orc, orc.Index(ctx["ks"], pairs=pairs, ntx=ctx["tx"].ntx)


def parity_sample(ctx, threads):
    """The sample through the oracle from FASTQ text, bit-exact against the GPU's export; returns
    (verdict, oracle index, FASTQ bytes, oracle seconds)."""
    orc, oi = oracle_index(ctx)
    m, L = ctx["m"], ctx["L"]
    fq = synth.fastq_bytes(ctx["bases"][:m * L], L)
    tc = time.perf_counter()
    cout = orc.fastq_map(oi, fq, nthreads=threads, outputs=True, hcap=64, ccap=64)
    dt = time.perf_counter() - tc
    bad = parity_check(ctx["gout"], ctx["gtot"], cout, len(ctx["ks"]))
    verdict = ("bit-exact, %d reads (status, retained-hash sets, candidate lists, per-transcript totals)" % m
               if not bad else "MISMATCH: " + "; ".join(bad))
    return verdict, (orc, oi), fq, dt


def release(ctx):
    ctx["sess"].free()
    ctx["index"].free()
    del ctx["d_reads"]
    ctx.clear()
    torch.cuda.empty_cache()


def main(args):
    cname = args.config or ("cfg3" if args.gpus == 1 else "cfg4")
    cfg = dict(CONFIGS[cname])
    if args.reads:
        cfg["reads"] = args.reads

    rank, world, local = sdist.world()
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    gpu = local % max(torch.cuda.device_count(), 1)  # one GPU per rank on a full node
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    line, ctx = measure(cname, cfg, args, rank, world, dev, gpu, args.cpu_reads)
    n, L = ctx["n"], ctx["L"]
    parity, cpu = None, None
    if rank == 0:
        P_thr, ncpu, share_how = cpu_share(args, world)
        parity, (orc, oi), fq, dt_p = parity_sample(ctx, P_thr)
        log("parity sample: %s" % parity)
        m = ctx["m"]
        # (every N: rank 0 times the same oracle path on its host-core share while the other ranks
        # wait at the barrier below)
        cpu = {"value": m / dt_p, "unit": "reads/s", "cores": P_thr, "kind": "port",
               "cpu_model": cpu_model(), "affinity_cpus": ncpu, "cores_derivation": share_how,
               "cores_note": "threads over read shards; the reference itself is single-threaded (see "
                             "single_core)",
               "sample": "first %d reads of rank 0's batch as FASTQ text (%d MB in RAM), same index: "
                         "oracle/oracle.c orc_fastq_map (record machine, is_valid_sequence, sketch, "
                         "sparse_chain, id map, totals), %d threads over read shards, %.1fs"
                         % (m, fq.size >> 20, P_thr, dt_p)}
        if not args.no_cpu_baseline:
            m1 = min(m, 1_000_000)
            fq1 = fq[:m1 * (fq.size // m)]
            tc = time.perf_counter()
            orc.fastq_map(oi, fq1, nthreads=1, outputs=False, totals=True)
            dt_1 = time.perf_counter() - tc
            cpu["single_core"] = {"value": m1 / dt_1, "cores": 1,
                                  "sample": "first %d reads, 1 thread, %.1fs" % (m1, dt_1)}
        cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
        if os.path.exists(cal):  # reference sparse_chain vs the oracle's, timed in the build container
            cpu["calibration"] = json.load(open(cal)).get("summary")
        del fq
    e2e = None
    if not args.no_end_to_end:
        try:
            e2e = end_to_end(ctx["index"], ctx["tx"].ntx, ctx["bases"], ctx["d_reads"].data_ptr(), n, L, ctx["sess"],
                             ctx["sp"], rank, world, dev, io_cfg=(args.io_threads, args.chunk_mb))
        except (OSError, skq.SkqError) as ex:  # (e.g. no room for the FASTQ file): the metric line still prints
            e2e = {"error": "%s: %s" % (type(ex).__name__, ex)}
        log("end to end: %s" % json.dumps(e2e))
    if world > 1:
        dist.barrier()
    release(ctx)

    # the other single-GPU configs of BASELINE.json, each with its own timed steps, roofline and
    # parity sample (never `value`): cfg2 (100 bp, 10k transcripts) and cfg5 (multi-k)
    extra = {}
    bad_extra = False
    if world == 1 and args.config is None and not args.reads and not args.no_extra_configs:
        for xc, xs in (("cfg2", 1_000_000), ("cfg5", 1_000_000)):
            xl, xctx = measure(xc, dict(CONFIGS[xc]), args, rank, world, dev, gpu, xs)
            xp, _, _, _ = parity_sample(xctx, cpu_share(args, world)[0])
            log("%s: %.3g reads/s, %.3f ms per step, parity sample: %s" % (xc, xl["value"], xl["ms_per_step"], xp))
            bad_extra |= xp.startswith("MISMATCH")
            xl.update(config={"workload": xc + ": " + CONFIGS[xc]["desc"], "reads_per_gpu": CONFIGS[xc]["reads"],
                              "read_len": CONFIGS[xc]["read_len"], "transcripts": CONFIGS[xc]["ntx"],
                              "ks": CONFIGS[xc]["ks"]},
                      steps=args.steps, warmup=args.warmup, settle_steps=xl.get("settle_steps"), parity_sample=xp)
            extra[xc] = xl
            release(xctx)

    if rank == 0:
        res = {
            "metric": METRIC, "value": line["value"], "unit": "reads/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": line["ms_per_step"], "higher_is_better": True,
            "settle_steps": line["settle_steps"],
            "settle_note": ("untimed batches before the warmup steps, until two groups of 5 take the same time "
                            "within 1.5 %: the memory clocks ramp over the first ~25 batches (DESIGN.md §6)"),
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": cname + ": " + cfg["desc"], "reads_per_gpu": n, "read_len": L,
                       "transcripts": cfg["ntx"], "ks": cfg["ks"], "sketch_fraction": "(double)0.05f",
                       "chain_fraction": 0.9, "parallelism": "read-sharded x%d, index replicated" % world
                       + (", 1 all-reduce of per-transcript totals per step" if world > 1 else "")},
            "roofline": line["roofline"],
            "path": line["path"],
            "parity_sample": parity,
            "cpu_baseline": cpu,
            "end_to_end": e2e,
        }
        if extra:
            res["configs"] = extra
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if (parity is not None and parity.startswith("MISMATCH")) or bad_extra:
        raise SystemExit(3)
    if e2e is not None and e2e.get("check") == "MISMATCH":
        raise SystemExit(4)


if __name__ == "__main__":
    main(_a)
