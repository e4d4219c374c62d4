#!/usr/bin/env python3
"""HBM traffic per read, per kernel, from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over bench.py.

usage: tools/traffic.py CONFIG FETCH_DIR WRITE_DIR OUT.json [KERNEL=STREAMED_BYTES_PER_READ ...]

Calibrated per profiles/r3_fetch_calibration.json (tools/micro/calib.hip on known byte counts, as
MI355X_MICROARCH.md "HBM [CDNA4]" requires for access widths other than wide streaming reads):
FETCH_SIZE tallies 64 B per memory-side read request; a streamed (coalesced) request moves 128 B,
a random 32-B entry gather is one 64-B request. So per kernel
    bytes = FETCH_SIZE(kB) * 1024 + STREAMED / 2 + WRITE_SIZE(kB) * 1024,
STREAMED being the bytes the kernel reads as coalesced streams (k_map1: the read bases, L per
read; given on the command line). Only the full-size dispatches of each kernel are used (largest
grid); the figure is divided by the grid's reads (one thread per read, 256 per workgroup),
giving bytes per read that bench.py scales to its launch.
"""
import collections
import csv
import glob
import json
import statistics
import sys

cfg, fdir, wdir, out = sys.argv[1:5]
streamed = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in sys.argv[5:]}


def per_read(d, counter):
    rows = collections.defaultdict(dict)
    full = {}  # dispatch -> full kernel name (template arguments included)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
            did = int(row["Dispatch_Id"])
            grid = int(row["Grid_Size"]) if "Grid_Size" in row else int(row["Grid_Size_X"])
            r = rows[name].setdefault(did, [grid, 0.0])
            r[1] += float(row["Counter_Value"])
            full[did] = row["Kernel_Name"].split("(")[0]
    res = {}
    for name, ds in rows.items():
        gmax = max(g for g, _ in ds.values())
        vals = [v / g for g, v in ds.values() if g == gmax]
        res[name] = (statistics.median(vals), len(vals), gmax)
    # several k slots: one k_map1 launch per k slot (template PASS = true), the last one FINAL;
    # a step's map is the run of full-size pass dispatches ending in a final one, summed
    # (bench.py names it "k_map1 xN passes")
    ds = rows.get("k_map1", {})
    if ds:
        gmax = max(g for g, _ in ds.values())
        groups, cur = collections.defaultdict(list), []
        for did in sorted(ds):
            g, v = ds[did]
            targs = full[did].split("<", 1)[1].rstrip(">").replace(" ", "").split(",") if "<" in full[did] else []
            if g != gmax or len(targs) < 5 or targs[3] != "true":
                continue
            cur.append(v / g)
            if targs[4] == "true":
                groups[len(cur)].append(sum(cur))
                cur = []
        for npass, vals in groups.items():
            res["k_map1 x%d passes" % npass] = (statistics.median(vals), len(vals), gmax)
    return res


fetch = per_read(fdir, "FETCH_SIZE")
write = per_read(wdir, "WRITE_SIZE")
kern = {}
for name in sorted(set(fetch) & set(write)):
    f, nf, g = fetch[name]
    w, nw, _ = write[name]
    sb = streamed.get(name, 0.0)
    kern[name] = {"fetch_size_bytes_per_read": f * 1024, "streamed_read_bytes_per_read": sb,
                  "fetch_bytes_per_read": f * 1024 + sb / 2, "write_bytes_per_read": w * 1024,
                  "hbm_bytes_per_read": f * 1024 + sb / 2 + w * 1024, "grid_threads": g,
                  "dispatches": [nf, nw]}
json.dump({"config": cfg, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --kernel-trace over "
           "bench.py", "calibration": "profiles/r3_fetch_calibration.json: bytes = FETCH_SIZE + streamed/2 + "
           "WRITE_SIZE (FETCH_SIZE tallies 64 B per request; streamed requests move 128 B, random 32-B "
           "gathers are 64-B requests)", "kernels": kern},
          open(out, "w"), indent=1)
print(json.dumps(kern, indent=1))
