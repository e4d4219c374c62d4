#!/bin/bash
# round 6: every GPU test + smoke, then the default bench line and its kernel trace.
# usage: tools/gpu_r6.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
t=${1:-r6}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $o/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { echo "tests failed"; tail -40 $o/tests.log; exit 1; }
  tail -3 $o/tests.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
  tail -1 $o/smoke.log
fi
timeout -k 10 500 python3 bench.py > $o/bench.json 2> $o/bench.err || { echo "bench failed"; tail -30 $o/bench.err; exit 1; }
python3 tools/bench_summary.py $o/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs > $o/stats_bench.json 2> $o/stats_bench.err || { echo "stats bench failed"; tail -20 $o/stats_bench.err; exit 1; }
python3 tools/trace_steps.py $o/stats/run_kernel_trace.csv > $o/trace_steps.txt 2>&1; tail -25 $o/trace_steps.txt
