#!/bin/bash
# round-6 first call: counter list + what binds k_map1 at cfg3 (bound set) on the round-5 tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r6a
mkdir -p $o
export PYTHONUNBUFFERED=1
timeout -s KILL 60 rocprofv3 -L > $o/avail.txt 2>&1 || echo "list failed"
tools/pmc.sh bound $o/bound --probes auto/chain --rounds 2 > $o/bound.log 2>&1 || { echo "bound failed"; tail -20 $o/bound.log; exit 1; }
python3 tools/pmc_bound.py $o/bound k_map1 10000000 > $o/bound.json && cat $o/bound.json
