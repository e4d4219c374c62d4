#!/bin/bash
# k_bin_packed with a small staging (beside the map instead of displacing it): parity, step time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "cfg3 or full_batch" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python3 tools/totals_steps.py --rounds 4 --steps 12 --variants "SKQ_BINP_CAP=0,SKQ_BINP_CAP=1,SKQ_BINP_CAP=0+SKQ_TOTALS_FORK=0" > $O/steps.log 2>&1 || { tail $O/steps.log; exit 1; }
grep -E "median|DIFFER" $O/steps.log
timeout -k 10 500 python3 tools/totals_steps.py --ntx 10000 --reads 1000000 --len 100 --steps 30 --rounds 4 --variants "SKQ_BINP_CAP=0,SKQ_BINP_CAP=1" > $O/steps2.log 2>&1 || { tail $O/steps2.log; exit 1; }
grep -E "median|DIFFER" $O/steps2.log
