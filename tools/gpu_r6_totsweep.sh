#!/bin/bash
# k_tot_small (chunks, range) sweep at cfg2 under a kernel trace (development). usage: tools/gpu_r6_totsweep.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SKQ_DEV=1
VARIANTS=${VARIANTS:-"64_10000 16_10000 32_10000 64_2560 128_5000"}
for v in $VARIANTS; do
  set -- ${v/_/ }
  export SKQ_TOT_CHUNKS=$1 SKQ_TOT_RANGE=$2
  timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr_$1_$2 -o run -- python3 bench.py --config cfg2 --no-cpu-baseline --no-end-to-end --steps 10 --warmup 2 --cpu-reads 20000 > $o/b_$1_$2.json 2> $o/b_$1_$2.err || { echo "run $v failed"; tail -20 $o/b_$1_$2.err; exit 1; }
  python3 - $o/tr_$1_$2/run_kernel_trace.csv "$v" <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_tot_small" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("chunks range %s: k_tot_small median %.1f us over %d" % (sys.argv[2], statistics.median(d[5:] or d), len(d)))
PY
done
