#!/bin/bash
# round 5: same-process A/Bs — L2 prefetch distance (SKQ_PREFETCH), the hashing loops
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5e
mkdir -p $O
(while sleep 50; do date >> $O/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
L=sketch-for-rna-seq_amd/lib/libskq.so
for d in 320 160 640; do
  timeout -k 10 300 python3 tools/abbench.py $L --env-b SKQ_PREFETCH=$d --rounds 20 > $O/ab_pf$d.log 2>&1 || { echo "ab pf $d rc=$?"; tail -20 $O/ab_pf$d.log; exit 1; }
  echo "== prefetch $d (B) vs off (A)"; tail -4 $O/ab_pf$d.log
done
timeout -k 10 300 python3 tools/abbench.py $L --env-b SKQ_PREFETCH=320 --acc --rounds 20 > $O/ab_pf320_acc.log 2>&1 || { echo "ab pf acc rc=$?"; tail -20 $O/ab_pf320_acc.log; exit 1; }
echo "== prefetch 320 (B) vs off (A), totals on"; tail -4 $O/ab_pf320_acc.log
timeout -k 10 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 20 > $O/ab_hash.log 2>&1 || { echo "ab hash rc=$?"; tail -20 $O/ab_hash.log; exit 1; }
echo "== round-4 hashing loop (B) vs pair terms (A)"; tail -4 $O/ab_hash.log
