#!/bin/bash
# kernel trace of tools/kbench.py (per-kernel durations incl. the slow paths)
set -o pipefail
t=${1:-r3w}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_kb -o run -- python3 tools/kbench.py --rounds 3 > gpurun_out/${t}_kb.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/${t}_kb.log; exit 1; }
grep -h "wall" gpurun_out/${t}_kb.log
python3 - "$t" <<'PY'
import csv, sys
t = sys.argv[1]
rows = list(csv.DictReader(open("gpurun_out/%s_kb/run_kernel_stats.csv" % t)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s calls %5s avg %10.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
