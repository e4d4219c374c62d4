#!/bin/bash
# TAB 4 with the query's pilot requested inside the hashing loop: parity, then A/B against TAB 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z
mkdir -p $O
PT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_parity.py -k "chain-compact" > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 900 $PT tests/test_gpu_scale.py -k "compact or tight or full_batch" > $O/scale.log 2>&1 || { echo "scale rc=$?"; tail -30 $O/scale.log; exit 1; }
tail -2 $O/scale.log
for c in cfg3 cfg2 cfg5; do
  timeout -k 10 400 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config $c --rounds 12 --env-b SKQ_CHAIN=2 > $O/ab_$c.log 2>&1 || { tail $O/ab_$c.log; exit 1; }
  echo "== $c (B = compact chained)"; tail -3 $O/ab_$c.log
done
