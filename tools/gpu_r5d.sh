#!/bin/bash
# round 5: totals binned after the map (k_bin_packed, candidate pairs by batch parity) — parity
# (every GPU test but the full-batch scale tests, then those), same-process A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d
mkdir -p $O
(while sleep 50; do date >> $O/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "not full_batch" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py -x -q --timeout 600 --timeout-method thread -k "full_batch" > $O/tests_full.log 2>&1 || { echo "full rc=$?"; tail -30 $O/tests_full.log; exit 1; }
tail -2 $O/tests_full.log
L=sketch-for-rna-seq_amd/lib/libskq.so
timeout -k 10 400 python3 tools/abbench.py $L --env-b SKQ_MAP_BINS=1 --acc --rounds 20 > $O/ab_bins.log 2>&1 || { echo "ab bins rc=$?"; tail -20 $O/ab_bins.log; exit 1; }
tail -5 $O/ab_bins.log
timeout -k 10 400 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 20 > $O/ab_hash.log 2>&1 || { echo "ab hash rc=$?"; tail -20 $O/ab_hash.log; exit 1; }
tail -5 $O/ab_hash.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > $O/counters.txt 2>&1 || echo "list-avail rc=$?"
wc -l $O/counters.txt
