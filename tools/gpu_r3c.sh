#!/bin/bash
# Round-3 call C: the partitioned map's k_part_b — padded bucket strides, partition size, L2 counters
set -o pipefail
t=${1:-r3c}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
run() {  # name, env..., -- kbench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/kbench.py --probes wide/part --rounds 3 > gpurun_out/${t}_${name}.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/${t}_${name}.log; exit 1; }
  grep -E "wall|totals" gpurun_out/${t}_${name}.log
}
run pad1 SKQ_PART_PAD=1
run pad0 SKQ_PART_PAD=0
run keys20k SKQ_PART_PAD=1 SKQ_PART_KEYS=20000
run bw128 SKQ_PART_PAD=1 SKQ_PART_BW=128
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_stats -o run -- python3 tools/kbench.py --probes wide/part --rounds 3 > gpurun_out/${t}_stats.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "stats ok"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d gpurun_out/${t}_pmc -o run -- python3 tools/kbench.py --probes wide/part --rounds 1 > gpurun_out/${t}_pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
echo "pmc ok"
