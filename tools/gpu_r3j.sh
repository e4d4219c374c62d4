#!/bin/bash
# chained tables: A/B timing, phase stamps, fabric request counters (wide vs wide/chain)
set -o pipefail
t=${1:-r3j}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 400 python -u tools/kbench.py --probes wide,wide/chain --rounds 5 --stamps > gpurun_out/${t}_kbench.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/${t}_kbench.log; exit 1; }
grep -v "^setup" gpurun_out/${t}_kbench.log | grep -v "start deciles"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d gpurun_out/${t}_pmc -o run -- python3 tools/kbench.py --probes wide,wide/chain --rounds 1 > gpurun_out/${t}_pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
echo "pmc ok"
