#!/bin/bash
# kernel-trace stats of one bench run: tools/gpu_stats.sh TAG [bench args]
set -o pipefail
tag=$1; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run \
  -- python3 bench.py --no-cpu-baseline --no-end-to-end --cpu-reads 200000 "$@" > gpurun_out/${tag}_stats.json 2> gpurun_out/${tag}_stats.err
