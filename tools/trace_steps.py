"""Print the last timed steps of a rocprofv3 kernel trace (gaps between dispatches, per queue).
usage: python3 tools/trace_steps.py TRACE.csv [N_STEPS]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nst = int(sys.argv[2]) if len(sys.argv) > 2 else 3
idx = [i for i, r in enumerate(rows) if "k_map1" in r["Kernel_Name"]]
ms = [int(rows[i]["Start_Timestamp"]) for i in idx]
d = [(b - a) / 1e3 for a, b in zip(ms, ms[1:])]
print("map-to-map us (last 12):", [round(x, 1) for x in d[-13:-1]])
i0 = idx[-nst - 2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:idx[-2]]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %8.1f %7.1f q%s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Kernel_Name"][:60]))
