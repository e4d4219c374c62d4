#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
t=${1:-r2y}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --cpu-reads 400000 > gpurun_out/${t}_bench.json 2> gpurun_out/${t}_bench.err &&
bash tools/gpu_stats.sh ${t} &&
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 --reads 2000000 --cpu-reads 100000 > gpurun_out/${t}_bench_n2.json 2> gpurun_out/${t}_bench_n2.err
