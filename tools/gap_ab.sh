#!/bin/bash
# A/B of the per-step launch gaps: bench lines at cfg2 / cfg3 with and without the per-kernel
# timing events and the totals fork, then a kernel trace of cfg2 without timing events
# usage: tools/gap_ab.sh TAG
set -o pipefail
t=${1:-gap}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env, args
  local nm=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs --steps 40 "$@" > $o/$nm.json 2> $o/$nm.err || { echo "$nm failed"; tail -20 $o/$nm.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-24s %.4f ms/step  %.3f G/s' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))" $o/$nm.json $nm | tee -a $o/summary.log
}
for rep in 1 2; do
  run c2_timing_$rep X=1 --config cfg2
  run c2_notiming_$rep X=1 --config cfg2 --no-kernel-timing
  run c2_nofork_notiming_$rep SKQ_TOTALS_FORK=0 --config cfg2 --no-kernel-timing
  run c3_timing_$rep X=1 --config cfg3
  run c3_notiming_$rep X=1 --config cfg3 --no-kernel-timing
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr2 -o run -- python3 bench.py --config cfg2 --no-cpu-baseline --no-end-to-end --no-extra-configs --no-kernel-timing --steps 20 > $o/tr2.json 2> $o/tr2.err || { echo "trace c2 failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr3 -o run -- python3 bench.py --config cfg3 --no-cpu-baseline --no-end-to-end --no-extra-configs --steps 20 > $o/tr3.json 2> $o/tr3.err || { echo "trace c3 failed"; exit 1; }
echo done
