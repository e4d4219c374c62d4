#!/bin/bash
# quick check: a subset of GPU tests, untraced bench lines (PLAIN) and bench kernel traces (TRACED, default cfg2 cfg3). usage: PLAIN="cfg..." TRACED="cfg..." tools/gpu_quick.sh TAG "pytest args"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
mkdir -p $o
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $o/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -u -m pytest $2 -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { echo "tests failed"; tail -40 $o/tests.log; exit 1; }
  tail -1 $o/tests.log
fi
for c in ${PLAIN:-}; do  # untraced bench lines
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-end-to-end > $o/p_$c.json 2> $o/p_$c.err || { echo "bench $c failed"; tail -20 $o/p_$c.err; exit 1; }
  python3 tools/bench_summary.py $o/p_$c.json | head -1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in ${TRACED:-cfg2 cfg3}; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --steps 20 > $o/b_$c.json 2> $o/b_$c.err || { echo "trace $c failed"; tail -20 $o/b_$c.err; exit 1; }
  python3 tools/bench_summary.py $o/b_$c.json | head -1
  python3 tools/trace_steps.py $o/tr_$c/run_kernel_trace.csv 2 > $o/steps_$c.txt 2>&1; head -9 $o/steps_$c.txt
done
