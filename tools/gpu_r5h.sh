#!/bin/bash
# compact chained tables (TAB 4) and the one-launch multi-k map (k_mapk): parity, then same-process
# A/Bs; the one-wave workgroup debug and the hashing-loop A/B; cfg2 batch-size sweep
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
step parity 600 $PT tests/test_gpu_parity.py -k "chain-compact or multi_k"
step scale 900 $PT tests/test_gpu_scale.py -k "chain-compact or cfg5"
step ab_cfg5_mapk 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config cfg5 --rounds 12 --env-b SKQ_MAPK=0
step ab_cfg5_tab4 400 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config cfg5 --rounds 12 --env-b SKQ_CHAIN=2
step ab_cfg3 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --rounds 20 --env-b SKQ_CHAIN=2
step ab_cfg2 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config cfg2 --rounds 20 --env-b SKQ_CHAIN=2
step ab_cfg5_wpe5 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/wpe5/libskq.so --config cfg5 --rounds 12
step ab_cfg3_tab4_wpe5 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/wpe5/libskq.so --rounds 20 --chain 2
step nsweep2 300 python3 tools/nsweep.py --config cfg2
SKQ_LIB=$PWD/sketch-for-rna-seq_amd/lib/ab/wg64/libskq.so step dbg 200 python3 tools/dbg_wg64.py
step ab_hash 300 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/oldhash/libskq.so --rounds 30
