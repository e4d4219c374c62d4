#!/bin/bash
# two-wave k_map1 workgroups (single k and passes) against the product (four-wave single k,
# one-wave passes); and k_mapk in one-wave workgroups against the pass launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5y
mkdir -p $O
B=sketch-for-rna-seq_amd/lib/ab/wg128/libskq.so
for c in cfg3 cfg5 cfg2; do
  timeout -k 10 400 python3 tools/abbench.py $B --config $c --rounds 14 > $O/$c.log 2>&1 || { echo "$c rc=$?"; tail $O/$c.log; exit 1; }
  echo "== $c"; tail -4 $O/$c.log
done
timeout -k 10 400 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config cfg5 --rounds 12 --env-b SKQ_MAPK=1 > $O/mapk.log 2>&1 || { tail $O/mapk.log; exit 1; }
echo "== k_mapk (B) vs passes (A)"; tail -4 $O/mapk.log
