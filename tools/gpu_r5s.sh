#!/bin/bash
# totals kernels v2 against v1, same process (wall time of map + totals, serialized)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s2
mkdir -p $O
OLD=sketch-for-rna-seq_amd/lib/ab/totals1/libskq.so
timeout -k 10 300 python3 tools/abbench.py $OLD --acc --rounds 20 > $O/cfg3.log 2>&1 || { tail $O/cfg3.log; exit 1; }
tail -4 $O/cfg3.log
timeout -k 10 300 python3 tools/abbench.py $OLD --acc --config cfg2 --rounds 30 > $O/cfg2.log 2>&1 || { tail $O/cfg2.log; exit 1; }
tail -4 $O/cfg2.log
timeout -k 10 300 python3 tools/abbench.py $OLD --acc --config cfg5 --rounds 10 > $O/cfg5.log 2>&1 || { tail $O/cfg5.log; exit 1; }
tail -4 $O/cfg5.log
