#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
tag=${1:-k5}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "multi_k or random_reads or scale" > gpurun_out/${tag}_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_cfg5.json 2> gpurun_out/${tag}_cfg5.err
