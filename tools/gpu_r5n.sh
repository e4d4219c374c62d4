#!/bin/bash
# bench step time against the warm-up length, beside the step-time tool (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs --no-kernel-timing"
for w in 3 30 3 100; do
  timeout -k 10 300 $B --warmup $w --steps 20 > $O/b_w$w.log 2>&1 || { echo "bench rc=$?"; tail $O/b_w$w.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_w$w.log').read().strip().splitlines()[-1])
print('warmup $w: %.4f ms/step' % d['ms_per_step'])"
done
timeout -k 10 300 python3 tools/totals_steps.py --rounds 3 --steps 20 > $O/steps.log 2>&1 || exit 1
grep -E "round|median" $O/steps.log
