#!/bin/bash
# round 5: sketcher / CLI / chained-sharing tests, same-process A/B of the hashing loops,
# the counter list of this rocprofv3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c
mkdir -p $O
(while sleep 50; do date >> $O/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 900 python3 -u -m pytest tests/test_dropin.py tests/test_cli.py tests/test_rccl_gpu.py tests/test_dropin_ref.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 20 > $O/ab_hash.log 2>&1 || { echo "ab rc=$?"; tail -20 $O/ab_hash.log; exit 1; }
tail -6 $O/ab_hash.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > $O/counters.txt 2>&1 || echo "list-avail rc=$?"
wc -l $O/counters.txt
