#!/bin/bash
# the record call's second half: the N > 1 rehearsal (2 ranks on one GPU over gloo) and cfg4's
# per-GPU shard on one GPU. usage: tools/gpu_record2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
t=${1:-r5r}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $o/hb2.log; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 500 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 > $o/bench_g2_gloo.json 2> $o/bench_g2_gloo.err || { echo "g2 failed"; tail -20 $o/bench_g2_gloo.err; exit 1; }
tail -c 400 $o/bench_g2_gloo.json; echo
timeout -k 10 500 python3 bench.py --config cfg4 --steps 10 --warmup 3 --no-extra-configs > $o/bench_cfg4_1gpu.json 2> $o/bench_cfg4_1gpu.err || { echo "cfg4 failed"; tail -20 $o/bench_cfg4_1gpu.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$o/bench_cfg4_1gpu.json').read().strip().splitlines()[-1])
print('cfg4 1gpu %.3f G/s %.4f ms frac %.4f e2e %s' % (d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['end_to_end']['reads_per_s']))"
