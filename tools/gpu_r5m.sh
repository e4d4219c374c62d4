#!/bin/bash
# does the bench's per-kernel timing (HIP events in the timed steps) cost step time? same box:
# bench.py with and without the events, the step-time tool, the kernel bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m
mkdir -p $O
step() {
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.log 2>&1
    local rc=$?
    echo "== $n rc=$rc"; grep -E "median|wall|\"value\"" $O/$n.log | cut -c1-400
    if [ $rc -ne 0 ]; then tail -5 $O/$n.log; exit $rc; fi
}
B="python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs --steps 20"
step bench_t 300 $B
step bench_nt 300 $B --no-kernel-timing
step bench_t2 300 $B
step bench_nt2 300 $B --no-kernel-timing
step steps 300 python3 tools/totals_steps.py --rounds 3 --steps 12
step kb 300 python3 tools/kbench.py --probes wide/chain --rounds 5
for f in bench_t bench_nt bench_t2 bench_nt2; do python3 -c "
import json,sys
d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1])
print('$f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms/step', 'k_map1', d['roofline'].get('avg_launch_ms'))
"; done
