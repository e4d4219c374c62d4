#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g
mkdir -p $O
SKQ_LIB=$PWD/sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so timeout -k 10 200 python3 tools/dbg_wg64.py > $O/dbg.log 2>&1; echo "dbg rc=$?"; tail -12 $O/dbg.log
timeout -k 10 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so --rounds 30 > $O/ab_wg64.log 2>&1; echo "ab rc=$?"
echo "== one-wave workgroups (B) vs four-wave (A)"; tail -5 $O/ab_wg64.log
timeout -k 10 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 30 > $O/ab_hash.log 2>&1 || { echo "ab hash rc=$?"; tail -20 $O/ab_hash.log; exit 1; }
echo "== round-4 hashing loop (B) vs v2 (A)"; tail -4 $O/ab_hash.log
