#!/bin/bash
# compact tables: parity (compact modes), then the bench in compact and wide mode (same box)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${1:-r2b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compact or scale" > gpurun_out/${tag}_tests.log 2>&1 &&
for cfg in cfg3 cfg5; do
  for pm in compact wide; do
    SKQ_PROBE=$pm timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_${cfg}_$pm.json 2> gpurun_out/${tag}_${cfg}_$pm.err || exit 1
  done
done
