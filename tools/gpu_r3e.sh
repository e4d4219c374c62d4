#!/bin/bash
# Round-3 call E: the chained tables — parity, scale parity, A/B against k_map1 with a kernel trace.
set -o pipefail
t=${1:-r3e}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chain" > gpurun_out/${t}_parity.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${t}_parity.log; exit 1; }
tail -2 gpurun_out/${t}_parity.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "chain" > gpurun_out/${t}_scale.log 2>&1 || { echo "scale failed"; tail -40 gpurun_out/${t}_scale.log; exit 1; }
tail -2 gpurun_out/${t}_scale.log
timeout -k 10 400 python -u tools/kbench.py --probes wide,wide/chain --rounds 5 > gpurun_out/${t}_kbench.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/${t}_kbench.log; exit 1; }
grep -v "^setup" gpurun_out/${t}_kbench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_stats -o run -- python3 tools/kbench.py --probes wide/chain --rounds 3 > gpurun_out/${t}_stats.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "stats ok"
