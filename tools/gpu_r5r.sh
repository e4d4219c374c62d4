#!/bin/bash
# totals kernels v2 (k_bin_packed over wave regions, k_bin_sum two segments in flight): every GPU
# test, then the step time and the serialized kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5r2
mkdir -p $O
bash tools/gpu_tests.sh r5r2 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 tools/totals_steps.py --rounds 3 --steps 12 --variants "SKQ_TOTALS_FORK=1,SKQ_TOTALS_FORK=0,SKQ_MAP_BINS=1+SKQ_TOTALS_FORK=0" > $O/steps.log 2>&1 || { tail $O/steps.log; exit 1; }
grep -E "median|DIFFER" $O/steps.log
SKQ_TOTALS_FORK=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/totals_steps.py --rounds 1 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 -c "
import csv
for row in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print('%-60s %6s %.4f' % (row['Name'][:60], row['Calls'], float(row['AverageNs'])/1e6))
" | head -8
