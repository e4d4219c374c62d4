#!/bin/bash
# Round-3 GPU call: the GPU tests, the default bench line, a 2-rank rehearsal of the N > 1 path
# (gloo on the one GPU, with the end-to-end leg), and the FETCH/WRITE/RDREQ calibration passes.
# usage: tools/gpu_round3.sh TAG [skip-tests]
set -o pipefail
t=${1:-r3}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${t}_tests.log; exit 1; }
  tail -3 gpurun_out/${t}_tests.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/${t}_bench.json 2> gpurun_out/${t}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${t}_bench.err; exit 1; }
echo "bench ok"
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --reads 2000000 --steps 5 --warmup 2 > gpurun_out/${t}_bench_g2.json 2> gpurun_out/${t}_bench_g2.err || { echo "bench g2 failed"; tail -20 gpurun_out/${t}_bench_g2.err; exit 1; }
echo "bench g2 ok"
for grp in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/${t}_calib_$tag -o run -- ./tools/micro/calib > gpurun_out/${t}_calib_$tag.log 2>&1 || { echo "calib $tag failed"; exit 1; }
done
echo "calib ok"
