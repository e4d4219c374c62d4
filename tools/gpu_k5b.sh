#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
tag=${1:-k5b}
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_cfg5.json 2> gpurun_out/${tag}_cfg5.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --cpu-reads 200000 > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
