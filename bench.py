#!/usr/bin/env python3
"""bench.py — reads/s of the quant hot path (FracMinHash sketch + sparse chain) on MI355X.

Workload (BASELINE.json configs[2], the metric's config): synthetic 150 bp forward-strand reads
against a ~200k-transcript GENCODE-scale synthetic index, k = 31, sketch fraction (double)0.05f,
chain fraction 0.9. One step = one pass of the hot path (k_sketch, k_probe, k_count, slow paths included)
over one batch of `--reads` reads already resident in HBM, plus — when N > 1 — the one RCCL
all-reduce of the per-transcript totals (reads, score) over xGMI.

One process per GPU (torch.distributed.run); reads are sharded (each rank its own seeded batch,
weak scaling), the index is replicated. rank 0 prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch  # first: libskq.so then binds to torch's HIP runtime (one runtime per process)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sketch-for-rna-seq_amd"))
import skq  # noqa: E402
from skq import dist as sdist  # noqa: E402
from skq import synth  # noqa: E402

METRIC = "reads/sec (quant, 150 bp, k=31) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GATHER_CEIL_GPS = 48.1  # random 32-B gathers per ns from an 8 GiB table (profiles/r1_gather_bench.log)

CONFIGS = {
    "cfg2": dict(ntx=10_000, reads=1_000_000, read_len=100, ks=[31],
                 desc="synthetic 1M x 100 bp reads vs 10k-transcript index, k=31"),
    "cfg3": dict(ntx=200_000, reads=10_000_000, read_len=150, ks=[31],
                 desc="synthetic 10M x 150 bp reads/GPU vs ~200k-transcript index, k=31"),
    "cfg5": dict(ntx=200_000, reads=10_000_000, read_len=150, ks=[21, 25, 31],
                 desc="synthetic 10M x 150 bp reads/GPU vs ~200k-transcript index, k={21,25,31}"),
}


def log(*a):
    print("[bench r%s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def per_read_stats(sess, tables, ks, n):
    """h (retained hashes, summed over k), P (postings touched), C (candidates) per read, from
    an export of the current results (deterministic given the inputs)."""
    out = sess.export()
    nk = len(ks)
    ho = out["hash_offs"].astype(np.int64)
    hs = out["hashes"]
    P = 0
    for i, k in enumerate(ks):
        keys, offs, _ = tables[k]
        # gather the k-slot-i hashes of every read
        starts = ho[i:-1:nk]
        ends = ho[i + 1::nk]
        lens = ends - starts
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        x = hs[idx]
        pos = np.searchsorted(keys, x)
        pos = np.minimum(pos, len(keys) - 1)
        hit = keys[pos] == x
        P += int((offs[pos + 1].astype(np.int64) - offs[pos].astype(np.int64))[hit].sum())
    h = len(hs) / n
    return dict(h=h, P=P / n, C=len(out["cand_tid"]) / n,
                ok=float((out["status"] == 0).mean()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--reads", type=int, default=0, help="reads per GPU (default: the config's)")
    ap.add_argument("--cpu-reads", type=int, default=2_000_000, help="CPU-baseline sample size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on one GPU)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.reads:
        cfg["reads"] = args.reads

    rank, world, local = sdist.world()
    gpu = local % max(torch.cuda.device_count(), 1)  # one GPU per rank on a full node
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    L, ks, n = cfg["read_len"], cfg["ks"], cfg["reads"]
    t0 = time.time()
    tx = synth.transcriptome(cfg["ntx"], seed=1)  # identical on every rank: replicated index
    tables = skq.build_tables(tx.seqs, tx.offs, ks, nthreads=16)
    index = skq.Index(ks, tx.ntx, tables, device=gpu)
    bases, _, _ = synth.reads(tx, n, L, seed=1000 + rank, err=0.001)  # rank's shard
    d_reads = torch.from_numpy(bases).to(dev)
    sess = skq.Session(index, n, L)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    totals = torch.zeros(2, tx.ntx, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    log("setup %.1fs: %d transcripts, %d reads x %d bp, index %s" % (
        time.time() - t0, tx.ntx, n, L, index.stats()))

    def step():
        sess.map(d_reads.data_ptr(), None, n, L, fixed_len=L, stream=sp)
        if world > 1:  # the one collective: per-transcript totals, summed over ranks (RCCL)
            sess.totals_to_device(totals[0].data_ptr(), totals[1].data_ptr(), stream=sp)
            sdist.allreduce_totals(totals)

    for _ in range(args.warmup):
        step()
    sess.check(sp)
    for kind in range(4):
        sess.kernel_time(kind)
    sess.enable_timing(True)
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
    # (total ms, launches): sketch, probe, count, totals (k_bin_sum + fold)
    kt = [sess.kernel_time(kind) for kind in range(4)]
    elapsed = sdist.max_over_ranks(elapsed, device=dev)  # the slowest rank's time

    # per-read workload figures on a 1M-read slice of this rank's batch
    ns = min(n, 1_000_000)
    sess.map(d_reads.data_ptr(), None, ns, L, fixed_len=L, stream=sp, accumulate=False)
    st = per_read_stats(sess, tables, ks, ns)
    h, P, Cn = st["h"], st["P"], st["C"]
    nk = len(ks)
    # algorithmic bytes per read, per kernel (DESIGN.md "Roofline"); an index lookup is priced at
    # the 8 B (key, list offset) it needs, a posting at its 4 B tid
    fused = kt[1][1] == 0  # no k_probe launches: the sketch kernel probed (direct/rank table)
    # wide tables, one k: skq_map runs ONE kernel (k_map1: sketch + entry gathers + count), timed
    # as kind 0 with no separate count launches
    map1 = kt[2][1] == 0 and kt[0][1] > 0
    # the count kernel: k_count3 (32-bit keys, bins the totals) unless ids need > 22 bits
    count_name = "k_count3" if tx.ntx <= (1 << 22) and os.environ.get("SKQ_VARIANT") != "4" else "k_count"
    b_chain = 4 * P + 4 + 8 * Cn + 4 * Cn  # postings in, candidates + count + binned totals out
    b_kern = {
        # read bases in; retained hashes, per-k counts, status out (+ when fused: one lookup per
        # hash, list offsets and the slow flag out)
        "k_sketch": L + 4 * h + 4 * nk + 1 + ((8 * h + 4 * h + 1) if fused else 0),
        # status + counts + hashes in, one lookup per hash, list offsets + slow flag out
        "k_probe": 1 + 4 * nk + 4 * h + 8 * h + 4 * h + 1,
        # status + flag + counts + list offsets in, postings, candidates (tid, score) + count out,
        # and each candidate's 4 B binned (tid, score) for the totals
        count_name: 2 + 4 * nk + 4 * h + 4 * P + 4 + 8 * Cn + 4 * Cn,
        # binned candidates in (4 B each), per-transcript sums out (amortised: 16 B x ntx / n)
        "totals": 4 * Cn + 16.0 * tx.ntx / n,
    }
    fused_name = "k_map1" if nk == 1 else "k_mapk"  # (k_mapk: 2..4 k slots)
    if map1:  # the fused kernel: read in, one lookup per hash, postings, hashes + candidates out
        b_kern = {fused_name: L + 1 + 4 * nk + 4 * h + 8 * h + b_chain, "totals": b_kern["totals"]}
    b_path = L + 8 * h + 4 * P + 4 * h + 8 * Cn         # SURVEY.md §8d formula
    names = (fused_name if map1 else "k_sketch", "k_probe", count_name, "totals")
    avg = {name: ms / cnt for name, (ms, cnt) in zip(names, kt) if cnt}
    kname = max(avg, key=avg.get)                       # dominant kernel
    achieved = n * b_kern[kname] / (avg[kname] * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    if os.path.exists(tf):                               # PMC FETCH/WRITE passes (tools/traffic.py)
        tr = json.load(open(tf))
        if kname in tr.get("kernels", {}):
            traffic = tr["kernels"][kname]["hbm_bytes_per_read"] * n
    # the bound that binds the lookups: random fabric requests, not bytes. k_map1
    # issues one random 32-B entry gather per retained hash; tools/micro/gather_bench measures the
    # chip's rate for exactly that access (pair-cooperative 32-B gathers, 8 GiB table).
    requests = None
    if map1:
        rps = n * h / (avg[kname] * 1e-3) / 1e9
        requests = {"random_per_read": h, "achieved": rps, "ceiling": GATHER_CEIL_GPS, "unit": "G/s",
                    "frac": rps / GATHER_CEIL_GPS,
                    "ceiling_source": "tools/micro/gather_bench: random pair-cooperative 32-B gathers, 8 GiB table"}
    total_reads = n * world * args.steps
    value = total_reads / elapsed

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import orc  # the CPU oracle: baseline only, never the measured path
        keys, offs, tids = tables[ks[0]]
        pairs = []
        for k in ks:
            keys, offs, tids = tables[k]
            pairs.append((np.repeat(keys, np.diff(offs.astype(np.int64))), tids))
        oi = orc.Index(ks, pairs=pairs, ntx=tx.ntx)
        m = min(args.cpu_reads, n)
        ro = np.arange(0, (m + 1) * L, L, dtype=np.uint64)
        tc = time.perf_counter()
        orc.lib().orc_map_batch_count(oi.h, orc.ptr(bases), orc.ptr(ro), m, orc.threshold(), 0.9)
        dt = time.perf_counter() - tc
        cpu = {"value": m / dt, "unit": "reads/s", "cores": 1, "kind": "port",
               "sample": "first %d reads of the same batch (in RAM), same index, oracle/oracle.c "
                         "single-threaded, %.1fs" % (m, dt)}

    if rank == 0:
        res = {
            "metric": METRIC, "value": value, "unit": "reads/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": args.config + ": " + cfg["desc"], "reads_per_gpu": n, "read_len": L,
                       "transcripts": tx.ntx, "ks": ks, "sketch_fraction": "(double)0.05f",
                       "chain_fraction": 0.9, "parallelism": "read-sharded x%d, index replicated" % world
                       + (", 1 all-reduce of per-transcript totals per step" if world > 1 else "")},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes": n * b_kern[kname], "avg_launch_ms": avg[kname],
                         "requests": requests,
                         # the PMC bytes per launch over the same launch time: every random entry
                         # gather moves a whole 128-B line
                         "traffic_GBps": traffic / (avg[kname] * 1e-3) / 1e9 if traffic else None},
            "path": {"bytes_per_read": b_path, "probe": (fused_name + " (sketch + wide-entry gathers + count fused)" if map1 else
                                                "fused in k_sketch" if fused else "k_probe"),
                     "index": index.stats(), "achieved_GBps": value / world * b_path / 1e9,
                     "frac": value / world * b_path / 1e9 / HBM_PEAK_GBS,
                     "kernel_ms": avg, "kernel_bytes_per_read": b_kern, "h": h, "P": P, "C": Cn},
            "cpu_baseline": cpu,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
