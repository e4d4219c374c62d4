#!/bin/bash
# Named variants of development switches (SKQ_DEV=1) at cfg3 (or CFG): an untraced bench
# line each, then kernel-trace medians of the map and the tail kernels for those named in TRACE
# (round 6: the totals binning's grouping and the CU-masked side stream, profiles/r6_bin_group_ab.log).
# usage: tools/gpu_variants.sh TAG "name:VAR=V,VAR=V name2:..."   (TRACE="name ..." to trace some)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
export PYTHONUNBUFFERED=1
run() {  # name spec out [extra bench args]
  local spec=$2
  ( export SKQ_DEV=1; IFS=','; for kv in $spec; do [ -n "$kv" ] && export "$kv"; done; unset IFS; shift 3; "$@" )
}
for v in $2; do
  name=${v%%:*}; spec=${v#*:}
  run $name "$spec" x timeout -k 10 200 python3 bench.py --config ${CFG:-cfg3} --no-cpu-baseline --no-end-to-end > $o/$name.json 2> $o/$name.err || { echo "$name failed"; tail -5 $o/$name.err; exit 1; }
  echo -n "$name: "; python3 tools/bench_summary.py $o/$name.json | head -1 | cut -c1-110
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $2; do
  name=${v%%:*}; spec=${v#*:}
  case " ${TRACE:-} " in *" $name "*) ;; *) continue ;; esac
  run $name "$spec" x timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr_$name -o run -- python3 bench.py --config ${CFG:-cfg3} --no-cpu-baseline --no-end-to-end --steps 10 > $o/t_$name.json 2> $o/t_$name.err || { echo "trace $name failed"; exit 1; }
  python3 - $o/tr_$name/run_kernel_trace.csv $name <<'PY'
import csv, sys, statistics, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("k_bin_packed", "k_bin_sum", "k_map1", "k_slow_wave"):
        if k in n and int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0) > 4096:
            d[n.split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print("%s %-40s median %.1f us over %d" % (sys.argv[2], k, statistics.median(v[-10:]), len(v)))
PY
done
