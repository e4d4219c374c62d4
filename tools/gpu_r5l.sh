#!/bin/bash
# totals parameters at cfg3 and cfg2: bucket bits, k_bin_sum workgroups, fork, bins in the map
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l
mkdir -p $O
step() {
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.log 2>&1
    local rc=$?
    echo "== $n rc=$rc"; grep -E "median|DIFFER" $O/$n.log
    if [ $rc -ne 0 ]; then tail -5 $O/$n.log; exit $rc; fi
}
V="SKQ_BIN_BITS=13,SKQ_BIN_BITS=13+SKQ_BIN_WGS=1024,SKQ_BIN_BITS=12+SKQ_BIN_WGS=1024,SKQ_BIN_BITS=12+SKQ_BIN_WGS=2048,SKQ_BIN_BITS=11+SKQ_BIN_WGS=2048,SKQ_BIN_BITS=11+SKQ_BIN_WGS=4096,SKQ_BIN_BITS=12+SKQ_BIN_WGS=2048+SKQ_MAP_BINS=1+SKQ_TOTALS_FORK=0,SKQ_BIN_BITS=13+SKQ_MAP_BINS=1+SKQ_TOTALS_FORK=0"
step cfg3 500 python3 tools/totals_steps.py --rounds 3 --steps 12 --variants "$V"
step cfg2 400 python3 tools/totals_steps.py --ntx 10000 --reads 1000000 --len 100 --steps 30 --rounds 3 --variants "$V"
