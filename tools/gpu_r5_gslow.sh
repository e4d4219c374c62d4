#!/bin/bash
# k_general_slow: every GPU test + smoke, then same-process A/B against the two-launch tail
# (SKQ_GENERAL_SLOW=0 in B) at cfg2 / cfg3 with totals, then bench lines without timing events
set -o pipefail
t=${1:-gslow}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_tests.sh $t || exit 1
L=sketch-for-rna-seq_amd/lib/libskq.so
for c in cfg2 cfg3; do
  timeout -k 10 200 python3 tools/abbench.py $L --config $c --acc --rounds 20 --env-b SKQ_GENERAL_SLOW=0 > $o/ab_$c.log 2>&1 || { echo "ab $c failed"; tail -20 $o/ab_$c.log; exit 1; }
  tail -4 $o/ab_$c.log
done
for c in cfg2 cfg3; do
  timeout -k 10 120 python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --no-extra-configs --steps 40 > $o/b_$c.json 2> $o/b_$c.err || { echo "bench $c failed"; tail -20 $o/b_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%s %.4f ms/step  %.3f G/s' % (sys.argv[2], d['ms_per_step'], d['value']/1e9))" $o/b_$c.json $c
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $o/tr2 -o run -- python3 bench.py --config cfg2 --no-cpu-baseline --no-end-to-end --no-extra-configs --no-kernel-timing --steps 20 > $o/tr2.json 2> $o/tr2.err || { echo "trace c2 failed"; exit 1; }
echo done
