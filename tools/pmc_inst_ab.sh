#!/bin/bash
# Instruction counts of k_map1 per SKQ_ABLATE value and probe (development): one --pmc pass per
# (probe, value) over tools/kbench.py; the deltas between values price each phase.
# usage: tools/pmc_inst_ab.sh OUT "PROBES" "VALUES"   e.g. tools/pmc_inst_ab.sh gpurun_out/ia "wide wide/chain" "0 2 4 32"
set -u
out=$1 probes=$2 vals=$3
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for pr in $probes; do
  for v in $vals; do
    tag=$(echo "$pr" | tr '/' '_')_$v
    SKQ_DEV=1 SKQ_ABLATE=$v timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$out/$tag/p1" -o run -- python3 tools/kbench.py --probes "$pr" --rounds 2 > "$out/$tag.log" 2>&1 || { echo "pass $tag failed rc=$?"; tail -5 "$out/$tag.log"; exit 1; }
    echo "== $tag"; python3 tools/pmc_summary.py "$out/$tag" | grep -A12 "k_map1"
  done
done
