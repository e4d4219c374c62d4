#!/bin/bash
# A/B of the totals binning's grouping at cfg3 (development: SKQ_BIN_G map workgroups per binned
# region, SKQ_BIN_GS lanes per region in k_bin_sum4): untraced bench lines, then kernel-trace medians
# of the tail kernels. usage: tools/gpu_bin_g.sh TAG ["G_GS ..."]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
export PYTHONUNBUFFERED=1
V=${2:-"4_4 8_4 8_8 4_8 1_4 4_4 8_4 8_8"}
for v in $V; do
  g=${v%_*}; gs=${v#*_}
  SKQ_DEV=1 SKQ_BIN_G=$g SKQ_BIN_GS=$gs timeout -k 10 200 python3 bench.py --config cfg3 --no-cpu-baseline --no-end-to-end > $o/g$v.json 2> $o/g$v.err || { echo "$v failed"; tail -5 $o/g$v.err; exit 1; }
  echo -n "G_GS=$v: "; python3 tools/bench_summary.py $o/g$v.json | head -1 | cut -c1-120
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${TRACE:-4_4 8_4}; do
  g=${v%_*}; gs=${v#*_}
  SKQ_DEV=1 SKQ_BIN_G=$g SKQ_BIN_GS=$gs timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr_g$v -o run -- python3 bench.py --config cfg3 --no-cpu-baseline --no-end-to-end --steps 10 > $o/tg$v.json 2> $o/tg$v.err || { echo "trace $v failed"; exit 1; }
  python3 - $o/tr_g$v/run_kernel_trace.csv $v <<'PY'
import csv, sys, statistics, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("k_bin_packed", "k_bin_sum", "k_map1", "k_slow_wave"):
        if k in n and int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0) > 4096:
            d[n.split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print("G_GS=%s %-40s median %.1f us over %d" % (sys.argv[2], k, statistics.median(v[-10:]), len(v)))
PY
done
