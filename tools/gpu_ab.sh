#!/bin/bash
# Same-box A/B over one environment switch (one gpurun call): for each value, one run of
#   bench   : bench.py [ARGS] (no cpu baseline)            -> value, ms/step, k_map1 ms, frac, e2e
#   kbench  : tools/kbench.py [ARGS]                       -> its wall / per-kernel lines
#   trace   : bench.py [ARGS] under rocprofv3 --kernel-trace -> tools/trace_summary.py
# (runs with SKQ_DEV=1: the library reads its development switches only then)
# usage: tools/gpu_ab.sh TAG bench|kbench|trace VAR "V1 V2 ..." [ARGS...]
#   e.g. tools/gpu_ab.sh binbits bench SKQ_BIN_BITS "13 12 11 13" --steps 20 --no-end-to-end
set -o pipefail
t=$1 kind=$2 var=$3 vals=$4
shift 4
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
for v in $vals; do
  f=gpurun_out/${t}_${var}_$v
  case $kind in
  bench)
    env SKQ_DEV=1 "$var=$v" timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $f.json 2> $f.err || { echo "bench failed"; tail -20 $f.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); e=d.get('end_to_end') or {}
print('$var=$v', 'value %.3f G/s' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'k_map1 %.3f' % d['roofline']['avg_launch_ms'],
      'frac %.4f' % d['roofline']['frac'], 'e2e', e.get('reads_per_s'))" ;;
  kbench)
    env SKQ_DEV=1 "$var=$v" timeout -k 10 400 python -u tools/kbench.py "$@" > $f.log 2>&1 || { echo "kbench failed"; tail -20 $f.log; exit 1; }
    echo "$var=$v"; grep -h "wall" $f.log ;;
  trace)
    env SKQ_DEV=1 "$var=$v" timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d ${f}_trace -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end "$@" > $f.json 2> $f.err || { echo "trace failed"; tail -20 $f.err; exit 1; }
    python3 tools/trace_summary.py $f.json ${f}_trace/run_kernel_trace.csv "$var=$v" ;;
  esac
done
