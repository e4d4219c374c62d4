#!/bin/bash
# parity + scale tests, then the cfg5 and cfg3 bench lines (no CPU baseline): tools/gpu_parity_benches.sh TAG
set -o pipefail
mkdir -p gpurun_out
tag=${1:-pb}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_cfg5.json 2> gpurun_out/${tag}_cfg5.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
