#!/bin/bash
# one-wave k_map1 workgroups (SKQ_MAP_WG=64 build) against four-wave ones, same process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5w
mkdir -p $O
B=sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so
for c in cfg3 cfg2 cfg5; do
  timeout -k 10 400 python3 tools/abbench.py $B --config $c --rounds 16 > $O/$c.log 2>&1 || { echo "$c rc=$?"; tail $O/$c.log; exit 1; }
  echo "== $c"; tail -4 $O/$c.log
done
