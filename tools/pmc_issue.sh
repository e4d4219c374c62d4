#!/bin/bash
# Issue-side PMC passes over tools/kbench.py: instruction mix, waits, LDS.
set -u
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_BRANCH" \
    "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o run -- python3 tools/kbench.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok"
done
