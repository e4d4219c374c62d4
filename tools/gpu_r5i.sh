#!/bin/bash
# the totals' cost per step: variants interleaved in one process, then kernel traces of the
# serialized (launch-stream) totals for per-kernel durations without overlap
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i
mkdir -p $O
step() {
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.log 2>&1
    local rc=$?
    echo "== $n rc=$rc"; tail -8 $O/$n.log
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step steps 400 python3 tools/totals_steps.py --rounds 3 --variants "SKQ_TOTALS_FORK=1,SKQ_TOTALS_FORK=0,SKQ_MAP_BINS=1,SKQ_MAP_BINS=1+SKQ_TOTALS_FORK=0,SKQ_BIN_BITS=12,SKQ_BIN_BITS=11+SKQ_TOTALS_FORK=0"
SKQ_TOTALS_FORK=0 step prof_nofork 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nofork -o run -- python3 tools/totals_steps.py --rounds 1
SKQ_TOTALS_FORK=0 SKQ_MAP_BINS=1 step prof_nofork_mapbins 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nofork_mapbins -o run -- python3 tools/totals_steps.py --rounds 1
for f in prof_nofork prof_nofork_mapbins; do echo "== $f"; python3 -c "
import csv,sys
for row in csv.DictReader(open('$O/$f/run_kernel_stats.csv')):
    print('%-60s %6s %.4f' % (row['Name'][:60], row['Calls'], float(row['AverageNs'])/1e6))
" | head -12; done
