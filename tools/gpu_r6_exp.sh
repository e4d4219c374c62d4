#!/bin/bash
# round 6 experiment call: kernel traces of the bench's steps per config, kbench (map alone vs with
# the totals) at cfg3. usage: tools/gpu_r6_exp.sh TAG [tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
t=${1:-r6x}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $o/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
if [ "$2" = "tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { echo "tests failed"; tail -40 $o/tests.log; exit 1; }
  tail -2 $o/tests.log
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in cfg2 cfg3 cfg5; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --steps 20 > $o/b_$c.json 2> $o/b_$c.err || { echo "trace $c failed"; tail -20 $o/b_$c.err; exit 1; }
  python3 tools/bench_summary.py $o/b_$c.json | head -1
  python3 tools/trace_steps.py $o/tr_$c/run_kernel_trace.csv 2 > $o/steps_$c.txt 2>&1; head -1 $o/steps_$c.txt
done
timeout -k 10 300 python3 tools/kbench.py --probes auto/chain --rounds 6 > $o/kbench_cfg3.log 2>&1 || { echo "kbench failed"; tail -20 $o/kbench_cfg3.log; exit 1; }
grep "wall" $o/kbench_cfg3.log
