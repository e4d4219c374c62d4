#!/bin/bash
# cfg5: the k=21 pass's raw capacity (16 at 3 sigma, 32 at 4 sigma): kernel trace + stats per setting
set -o pipefail
t=${1:-r3p}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
for sg in ${SIGMAS:-3 4}; do
  SKQ_PASS_SIGMAS=$sg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_s$sg -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-end-to-end > gpurun_out/${t}_s$sg.json 2> gpurun_out/${t}_s$sg.err || { echo "cfg5 failed"; tail -20 gpurun_out/${t}_s$sg.err; exit 1; }
  python3 - "$t" "$sg" <<'PY'
import csv, json, sys, collections
t, sg = sys.argv[1], sys.argv[2]
d = json.loads(open("gpurun_out/%s_s%s.json" % (t, sg)).read().strip().splitlines()[-1])
print("sigma", sg, "ms/step", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4))
k = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/%s_s%s/run_kernel_trace.csv" % (t, sg))):
    if r["Grid_Size_X"] in ("10000128",) or "slow" in r["Kernel_Name"] or "bin_sum" in r["Kernel_Name"]:
        k[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(k.items()):
    v2 = sorted(v)
    print("  %-48s n=%3d median %7.1f us" % (n, len(v), v2[len(v2) // 2]))
PY
done
