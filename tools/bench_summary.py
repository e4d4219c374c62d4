#!/usr/bin/env python3
"""One line per config of a bench.py JSON line: value, step, dominant kernel, fractions, parity.
usage: tools/bench_summary.py BENCH.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])


def line(name, x):
    r = x["roofline"]
    p = x.get("path", {})
    print("%s %.3f G reads/s, %.4f ms/step, %s %.4f ms, hbm frac %.4f, bound %s, fractions %s, slow %s, parity %s" % (
        name, x["value"] / 1e9, x["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"], r["bound"],
        {k: round(v, 3) for k, v in (r.get("fractions") or {}).items()}, p.get("slow_reads_per_batch"),
        str(x.get("parity_sample"))[:40]))


line("cfg3", d)
for c, x in (d.get("configs") or {}).items():
    line(c, x)
print("e2e", (d.get("end_to_end") or {}).get("reads_per_s"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
