#!/usr/bin/env python3
"""Vector / scalar / LDS instruction counts per read of the fused map, from rocprofv3 counter passes
(SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES over tools/kbench.py or bench.py), for
bench.py's second roofline (roofline.valu: the launch against the VALU issue peak).

A launch is a full batch of `--reads` reads. One k slot: every k_map1 dispatch of that size is one
launch. Several k slots: the pass dispatches (PASS kernels) of one batch are summed, a batch ending
at its FINAL pass. Per-read figures are the median over launches.

usage: tools/valu_counts.py PMC_DIR --reads 10000000 --config cfg3 --probe wide --chained 1 \
           [--measured "..."] > profiles/valu_cfg3.json
"""
import argparse
import collections
import csv
import glob
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("--reads", type=int, required=True)
ap.add_argument("--config", required=True)
ap.add_argument("--probe", default="wide")
ap.add_argument("--chained", type=int, default=1)
ap.add_argument("--measured", default="builder's rocprofv3 --pmc pass over tools/kbench.py")
a = ap.parse_args()

disp = collections.defaultdict(dict)  # dispatch id -> counter -> value (summed over XCD rows)
name = {}
grid = {}
for f in sorted(glob.glob(a.pmc_dir + "/**/run_counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        kn = row["Kernel_Name"]
        if "k_map1" not in kn:
            continue
        d = (f, int(row["Dispatch_Id"]))
        name[d] = kn
        grid[d] = int(row["Grid_Size"])
        c = row["Counter_Name"]
        disp[d][c] = disp[d].get(c, 0.0) + float(row["Counter_Value"])
full = (a.reads + 255) // 256 * 256


def targs(kn):  # k_map1<HCAP, MB, TAB, PASS, FINAL>
    t = [x.strip() for x in kn.split("<", 1)[1].split(">", 1)[0].split(",")]
    return t[3] == "true", t[4] == "true"


launches = []
acc = collections.Counter()
npass = 0
for d in sorted(disp):
    if not a.reads <= grid[d] < a.reads + 256:
        continue  # (the parity sample and other sizes; workgroups of 64 or 256 threads)
    is_pass, is_final = targs(name[d])
    if not is_pass:
        launches.append(dict(disp[d]))  # one k slot: this dispatch is the launch
        continue
    acc.update(disp[d])  # pass kernels: summed up to the batch's final pass
    npass += 1
    if is_final:
        launches.append(dict(acc))
        acc = collections.Counter()
if not launches:
    raise SystemExit("no full-size k_map1 launches in %s" % a.pmc_dir)
per = {}
for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"):
    vals = [x[c] for x in launches if c in x]
    if vals:
        per[c] = statistics.median(vals)
kname = "k_map1" if npass == 0 else "k_map1 x%d passes" % (npass // len(launches))
out = {
    "config": a.config, "probe": a.probe, "chained": bool(a.chained), "reads_per_launch": a.reads,
    "measured": a.measured, "launches": len(launches),
    "kernels": {kname: {
        "valu_per_read": per["SQ_INSTS_VALU"] / a.reads,
        "salu_per_read": per.get("SQ_INSTS_SALU", 0.0) / a.reads,
        "lds_per_read": per.get("SQ_INSTS_LDS", 0.0) / a.reads,
        "valu_per_wave": per["SQ_INSTS_VALU"] / per["SQ_WAVES"] if "SQ_WAVES" in per else None,
        "valu_per_launch": per["SQ_INSTS_VALU"],
        "waves_per_launch": per.get("SQ_WAVES"),
    }},
}
print(json.dumps(out, indent=1))
