#!/bin/bash
# ingest pipeline check + end-to-end figure; cfg5 kernel trace (the final pass's outliers)
set -o pipefail
t=${1:-r3m}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
SKQ_MAP1_OCC=1 timeout -k 10 300 python -u tools/kbench.py --rounds 5 > gpurun_out/${t}_kb_tight.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/${t}_kb_tight.log; exit 1; }
SKQ_MAP1_OCC=1 SKQ_MAP1_LOOSE=1 timeout -k 10 300 python -u tools/kbench.py --rounds 5 > gpurun_out/${t}_kb_loose.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/${t}_kb_loose.log; exit 1; }
grep -h "workgroups per CU\|k_map1\|ms" gpurun_out/${t}_kb_tight.log gpurun_out/${t}_kb_loose.log | tail -20
timeout -k 10 600 python -u -m pytest tests/test_ingest.py tests/test_cli.py tests/test_rccl_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${t}_tests.log; exit 1; }
tail -2 gpurun_out/${t}_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${t}_bench.json 2> gpurun_out/${t}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${t}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${t}_bench.json').read().strip().splitlines()[-1])
print('value', d['value']/1e9, 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
e=d['end_to_end']; print('e2e', e.get('reads_per_s'), e.get('pass_reads_per_s'), e.get('check'), e.get('em_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${t}_cfg5 -o run -- python3 bench.py --config cfg5 --no-cpu-baseline --no-end-to-end > gpurun_out/${t}_cfg5.json 2> gpurun_out/${t}_cfg5.err || { echo "cfg5 failed"; tail -20 gpurun_out/${t}_cfg5.err; exit 1; }
echo "cfg5 trace ok"
