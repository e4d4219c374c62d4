#!/bin/bash
# Round-2 record: GPU tests, the default bench line (with the CPU baseline), its rocprof
# kernel-trace stats and FETCH/WRITE passes (traffic), the cfg2 / cfg5 bench lines.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
t=r2i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/${t}_bench.json 2> gpurun_out/${t}_bench.err &&
bash tools/profile_round.sh ${t} &&
python3 tools/traffic.py cfg3 gpurun_out/${t}_FETCH_SIZE gpurun_out/${t}_WRITE_SIZE gpurun_out/${t}_traffic_cfg3.json > /dev/null &&
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > gpurun_out/${t}_bench_cfg5.json 2> gpurun_out/${t}_bench_cfg5.err &&
timeout -k 10 300 python -u bench.py --config cfg2 --no-cpu-baseline > gpurun_out/${t}_bench_cfg2.json 2> gpurun_out/${t}_bench_cfg2.err
