#!/bin/bash
# the full GPU suite on the product tree; the staged earlier-pass entries (an A/B build): its
# multi-k parity, then cfg5 against the product, same process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ac
mkdir -p $O
bash tools/gpu_tests.sh t5h || exit $?
S=$PWD/sketch-for-rna-seq_amd/lib/ab/staged/libskq.so
PT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
SKQ_LIB=$S timeout -k 10 900 $PT tests/test_gpu_parity.py -k "multi_k or k_slots or missing or five" > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
SKQ_LIB=$S timeout -k 10 900 $PT tests/test_gpu_scale.py -k "cfg5" > $O/scale.log 2>&1 || { echo "scale rc=$?"; tail -30 $O/scale.log; exit 1; }
tail -2 $O/scale.log
timeout -k 10 400 python3 tools/abbench.py $S --config cfg5 --rounds 12 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -4 $O/ab.log
