#!/bin/bash
# per-kernel times of the totals kernels v1 / v2, serialized (launch stream), alternating runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5t2
mkdir -p $O
OLD=$PWD/sketch-for-rna-seq_amd/lib/ab/totals1/libskq.so
for v in new old new old; do
  L=""; [ $v = old ] && L=$OLD
  SKQ_LIB=$L SKQ_TOTALS_FORK=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/totals_steps.py --rounds 1 > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  echo "== $v"; python3 -c "
import csv
for row in csv.DictReader(open('$O/$v/run_kernel_stats.csv')):
    if 'bin' in row['Name'] or 'k_map1' in row['Name']: print('%-40s %6s %.4f' % (row['Name'][:40], row['Calls'], float(row['AverageNs'])/1e6))
"
done
