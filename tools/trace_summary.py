#!/usr/bin/env python3
"""Summarise one bench.py line and its rocprofv3 kernel trace (development tool): ms/step, frac,
and the median duration of the map kernels and slow paths.

usage: tools/trace_summary.py BENCH_JSON KERNEL_TRACE_CSV [LABEL]"""
import collections
import csv
import json
import sys

line = open(sys.argv[1]).read().strip().splitlines()[-1]
d = json.loads(line)
label = sys.argv[3] if len(sys.argv) > 3 else ""
print(label, "ms/step", round(d["ms_per_step"], 3), "value", round(d["value"] / 1e9, 3), "G/s frac",
      round(d["roofline"]["frac"], 4))
k = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[2])):
    n = r["Kernel_Name"]
    if any(x in n for x in ("k_map1", "slow", "bin_sum", "fold")):
        k[n[:56]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(k.items()):
    v2 = sorted(v)
    print("  %-56s n=%3d median %8.1f us  max %8.1f" % (n, len(v), v2[len(v2) // 2], v2[-1]))
