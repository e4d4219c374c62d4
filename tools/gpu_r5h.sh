#!/bin/bash
# compact chained tables (TAB 4): parity, then same-process A/B against the chained wide tables;
# the one-wave workgroup debug and the hashing-loop A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5h
mkdir -p $O
step() {  # name seconds cmd...: stops the script after a crash, abort or time limit
    local n=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/$n.log 2>&1
    local rc=$?
    echo "== $n rc=$rc"; tail -6 $O/$n.log
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
    return 0
}
PT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
step parity 600 $PT tests/test_gpu_parity.py -k "chain-compact"
step scale 600 $PT tests/test_gpu_scale.py -k "chain-compact"
step ab_cfg3 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --rounds 20 --env-b SKQ_CHAIN=2
step ab_cfg2 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config cfg2 --rounds 20 --env-b SKQ_CHAIN=2
SKQ_LIB=$PWD/sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so step dbg 200 python3 tools/dbg_wg64.py
step ab_hash 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 30
step nsweep2 300 python3 tools/nsweep.py --config cfg2
step stamps2 300 python3 tools/kbench.py --ntx 10000 --reads 1000000 --len 100 --probes wide/chain --rounds 3 --stamps
