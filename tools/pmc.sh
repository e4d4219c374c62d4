#!/bin/bash
# PMC passes over tools/kbench.py (one counter group per rocprofv3 run, kernel-trace only).
# usage: tools/pmc.sh OUTDIR [kbench args...]
set -u
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
    "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
    "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o run -- python3 tools/kbench.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok: $grp"
done
