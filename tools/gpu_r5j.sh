#!/bin/bash
# the totals variants at cfg2 and cfg5 (cfg3: r5i)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j
mkdir -p $O
step() {
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.log 2>&1
    local rc=$?
    echo "== $n rc=$rc"; tail -5 $O/$n.log
    if [ $rc -ne 0 ]; then exit $rc; fi
}
V="SKQ_TOTALS_FORK=1,SKQ_TOTALS_FORK=0,SKQ_MAP_BINS=1,SKQ_MAP_BINS=1+SKQ_TOTALS_FORK=0"
step cfg2 300 python3 tools/totals_steps.py --ntx 10000 --reads 1000000 --len 100 --steps 30 --rounds 4 --variants "$V"
step cfg5 400 python3 tools/totals_steps.py --ks 21,25,31 --steps 5 --rounds 3 --variants "$V"
step cfg3 400 python3 tools/totals_steps.py --rounds 4 --variants "$V"
