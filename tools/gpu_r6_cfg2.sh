#!/bin/bash
# cfg2's step: kernel traces of the bench steps with the tail on the launch stream (default) and on
# the side stream (SKQ_SIDE_MIN=0). usage: tools/gpu_r6_cfg2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
mkdir -p $o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default side; do
  if [ $v = side ]; then export SKQ_DEV=1 SKQ_SIDE_MIN=0; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr_$v -o run -- python3 bench.py --config cfg2 --no-cpu-baseline --no-end-to-end --steps 20 > $o/b_$v.json 2> $o/b_$v.err || { echo "trace $v failed"; tail -20 $o/b_$v.err; exit 1; }
  python3 tools/bench_summary.py $o/b_$v.json | head -1
  python3 tools/trace_steps.py $o/tr_$v/run_kernel_trace.csv 2 > $o/steps_$v.txt 2>&1; head -14 $o/steps_$v.txt
done
