#!/bin/bash
# round 5, first call: LDS wrap check, k_map1 phase stamps (chained, current kernel), full-batch
# parity on the chained tables
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
(while sleep 50; do date >> gpurun_out/r5a_hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 60 tools/micro/lds_oob > gpurun_out/r5a_oob.log 2>&1 || { echo "oob rc=$?"; cat gpurun_out/r5a_oob.log; exit 1; }
cat gpurun_out/r5a_oob.log
timeout -k 10 400 python3 tools/kbench.py --probes wide/chain --rounds 3 --stamps > gpurun_out/r5a_stamps.log 2>&1 || { echo "kbench rc=$?"; tail -20 gpurun_out/r5a_stamps.log; exit 1; }
tail -30 gpurun_out/r5a_stamps.log
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_scale.py -x -v --timeout 900 --timeout-method thread -k full_batch > gpurun_out/r5a_fullbatch.log 2>&1
rc=$?
tail -15 gpurun_out/r5a_fullbatch.log
exit $rc
