#!/bin/bash
# batch-tail A/B (bench lines, timing events on as in the record): k_general_slow (SKQ_GENERAL_SLOW)
# and the late totals hand-off (SKQ_FORK_LATE), interleaved, then a cfg2 trace of the late hand-off
set -o pipefail
t=${1:-tail}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, env, args
  local nm=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs --steps 40 "$@" > $o/$nm.json 2> $o/$nm.err || { echo "$nm failed"; tail -20 $o/$nm.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-22s %.4f ms/step  %.3f G/s' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))" $o/$nm.json $nm | tee -a $o/summary.log
}
for rep in 1 2 3; do
  for c in cfg2 cfg3; do
    run ${c}_two_$rep "SKQ_GENERAL_SLOW=0 SKQ_FORK_LATE=0" --config $c
    run ${c}_gs_$rep "SKQ_GENERAL_SLOW=1 SKQ_FORK_LATE=0" --config $c
    run ${c}_gs_late_$rep "SKQ_GENERAL_SLOW=1 SKQ_FORK_LATE=1" --config $c
  done
done
SKQ_FORK_LATE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr2 -o run -- python3 bench.py --config cfg2 --no-cpu-baseline --no-end-to-end --no-extra-configs --no-kernel-timing --steps 20 > $o/tr2.json 2> $o/tr2.err || { echo "trace c2 failed"; exit 1; }
echo done
