#!/bin/bash
# round 5: pair-term hashing loop — parity, same-box A/B against the round-4 loop (SKQ_HASH_PAIR=0
# build), instruction counters of both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b
mkdir -p $O
(while sleep 50; do date >> $O/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
OLD=$PWD/sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "not full_batch" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/kbench.py --probes wide/chain --rounds 5 > $O/kb_new_$i.log 2>&1 || { echo "kb new rc=$?"; tail $O/kb_new_$i.log; exit 1; }
  SKQ_LIB=$OLD timeout -k 10 300 python3 tools/kbench.py --probes wide/chain --rounds 5 > $O/kb_old_$i.log 2>&1 || { echo "kb old rc=$?"; tail $O/kb_old_$i.log; exit 1; }
  grep -h "G reads/s" $O/kb_new_$i.log $O/kb_old_$i.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new old; do
  L=""; [ $v = old ] && L=$OLD
  SKQ_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_$v/p1 -o run -- python3 tools/kbench.py --probes wide/chain --rounds 2 > $O/pmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; tail -5 $O/pmc_$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py $O/pmc_$v | grep -A12 "k_map1"
done
