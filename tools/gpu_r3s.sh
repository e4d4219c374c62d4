#!/bin/bash
# k_map1 write-request experiment: drop the hash rows (1), the candidate rows (2), both (3)
set -o pipefail
t=${1:-r3s}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for d in 0 1 2 3 0; do
  SKQ_DBG_WRITES=$d timeout -k 10 300 python -u tools/kbench.py --rounds 5 > gpurun_out/${t}_d$d.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/${t}_d$d.log; exit 1; }
  echo "dbg $d"; grep -h "wall" gpurun_out/${t}_d$d.log
done
