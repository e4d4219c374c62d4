#!/bin/bash
# what warms up: bench steps after unrelated GPU work (clocks) or after small maps (tables)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5o
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs --no-kernel-timing --warmup 3 --steps 20"
for p in none matmul map1m none matmul map1m; do
  timeout -k 10 300 $B --preheat $p > $O/b_$p.log 2>&1 || { echo "bench rc=$?"; tail $O/b_$p.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$p.log').read().strip().splitlines()[-1])
print('preheat $p: %.4f ms/step' % d['ms_per_step'])"
done
