#!/bin/bash
# k_map1 change check: parity (probe modes, cfg3/cfg5 scale) then kbench timing
set -o pipefail
t=${1:-r3r}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_scale.py::test_cfg3_200k_transcripts_150bp" "tests/test_gpu_scale.py::test_cfg5_multi_k_200k_transcripts" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${t}_tests.log; exit 1; }
tail -2 gpurun_out/${t}_tests.log
timeout -k 10 300 python -u tools/kbench.py --rounds ${ROUNDS:-7} ${KB_ARGS:-} > gpurun_out/${t}_kb.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/${t}_kb.log; exit 1; }
grep -h "ms" gpurun_out/${t}_kb.log | tail -6
