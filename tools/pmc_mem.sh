#!/bin/bash
# Memory-side PMC passes over tools/kbench.py: fabric fetch/write, DRAM vs Infinity-Cache reads.
set -u
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o run -- python3 tools/kbench.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok"
done
