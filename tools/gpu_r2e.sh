#!/bin/bash
# slow wave path: full parity suite, then the bench (wide, default)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${1:-r2e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --cpu-reads 400000 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err &&
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_bench_cfg5.json 2> gpurun_out/${tag}_bench_cfg5.err
