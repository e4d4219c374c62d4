#!/bin/bash
# k_general_slow with one shared LDS region: every GPU test + smoke, a cfg3 kernel trace of the
# bench (timing events on, as in the record), then bench-line A/B against the two-launch tail
set -o pipefail
t=${1:-gslow2}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_tests.sh $t || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr3 -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs > $o/tr3.json 2> $o/tr3.err || { echo "trace c3 failed"; exit 1; }
run() {  # name, env, args
  local nm=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs --steps 40 "$@" > $o/$nm.json 2> $o/$nm.err || { echo "$nm failed"; tail -20 $o/$nm.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-22s %.4f ms/step  %.3f G/s' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))" $o/$nm.json $nm | tee -a $o/summary.log
}
for rep in 1 2 3; do
  for c in cfg2 cfg3; do
    run ${c}_two_$rep SKQ_GENERAL_SLOW=0 --config $c
    run ${c}_gs_$rep SKQ_GENERAL_SLOW=1 --config $c
  done
done
echo done
