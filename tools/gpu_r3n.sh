#!/bin/bash
# end-to-end ingest: pread threads x chunk size sweep (bench.py's end-to-end leg)
set -o pipefail
t=${1:-r3n}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IFS=, read -ra CF <<< "${CFGS:-8 64,16 64,16 128,12 32}"
for cfg in "${CF[@]}"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --io-threads $1 --chunk-mb $2 > gpurun_out/${t}_io$1_$2.json 2> gpurun_out/${t}_io$1_$2.err || { echo "bench failed"; tail -20 gpurun_out/${t}_io$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${t}_io$1_$2.json').read().strip().splitlines()[-1])
e=d['end_to_end']; print('io $1 chunk $2', round(e['reads_per_s']/1e6,1), [round(x/1e6,1) for x in e['pass_reads_per_s']], e['check'])"
done
