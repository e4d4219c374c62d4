#!/bin/bash
# every GPU test, then smoke(): tools/gpu_tests.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
t=${1:-tests}
O=gpurun_out/$t
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --durations=25 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -32 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -5 $O/smoke.log
exit $rc
