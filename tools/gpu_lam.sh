#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for lam in 5 10 16 24; do
  SKQ_CMP_LAMBDA=$lam SKQ_PROBE=compact timeout -k 10 300 python -u bench.py --no-cpu-baseline --cpu-reads 100000 --steps 6 > gpurun_out/lam_$lam.json 2> gpurun_out/lam_$lam.err || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --cpu-reads 100000 --steps 6 > gpurun_out/lam_wide.json 2> gpurun_out/lam_wide.err
