#!/bin/bash
# round 5: hashing loop v2 (16-entry terms, three-way XOR) and one-wave k_map1 workgroups —
# parity for both builds, same-process A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f
mkdir -p $O
(while sleep 50; do date >> $O/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "not full_batch" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SKQ_LIB=$PWD/sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "not full_batch" > $O/tests_wg64.log 2>&1 || { echo "tests wg64 rc=$?"; tail -30 $O/tests_wg64.log; exit 1; }
tail -2 $O/tests_wg64.log
timeout -k 10 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so --rounds 30 > $O/ab_wg64.log 2>&1 || { echo "ab wg64 rc=$?"; tail -20 $O/ab_wg64.log; exit 1; }
echo "== one-wave workgroups (B) vs four-wave (A)"; tail -4 $O/ab_wg64.log
timeout -k 10 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so --acc --rounds 30 > $O/ab_wg64_acc.log 2>&1 || { echo "ab wg64 acc rc=$?"; tail -20 $O/ab_wg64_acc.log; exit 1; }
echo "== one-wave workgroups (B) vs four-wave (A), totals on"; tail -4 $O/ab_wg64_acc.log
timeout -k 10 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 30 > $O/ab_hash.log 2>&1 || { echo "ab hash rc=$?"; tail -20 $O/ab_hash.log; exit 1; }
echo "== round-4 hashing loop (B) vs v2 (A)"; tail -4 $O/ab_hash.log
