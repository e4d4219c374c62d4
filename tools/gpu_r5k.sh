#!/bin/bash
# index kinds at cfg2 and cfg3 (wide, compact, each with and without chained tables), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
step() {
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.log 2>&1
    local rc=$?
    echo "== $n rc=$rc"; grep -E "wall|device_bytes|DIFFER" $O/$n.log | cut -c1-200
    if [ $rc -ne 0 ]; then tail -5 $O/$n.log; exit $rc; fi
}
step cfg2 400 python3 tools/kbench.py --ntx 10000 --reads 1000000 --len 100 --rounds 20 --probes wide/chain,wide,compact,compact/chain --acc-all
step cfg3 500 python3 tools/kbench.py --rounds 8 --probes wide/chain,wide,compact,compact/chain --acc-all
