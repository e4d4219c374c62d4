#!/bin/bash
# early k_slow_wave: cfg5 parity (late/early, full 2M batch) + multi-k parity modes, then cfg5 A/B
set -o pipefail
t=${1:-r3q}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -k "cfg5" tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${t}_tests.log; exit 1; }
tail -2 gpurun_out/${t}_tests.log
for ev in ${EARLY:-0 1}; do
  SKQ_EARLY_SLOW=$ev timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_e$ev -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-end-to-end > gpurun_out/${t}_e$ev.json 2> gpurun_out/${t}_e$ev.err || { echo "cfg5 failed"; tail -20 gpurun_out/${t}_e$ev.err; exit 1; }
  python3 tools/trace_summary.py gpurun_out/${t}_e$ev.json gpurun_out/${t}_e$ev/run_kernel_trace.csv "early=$ev"
done
