#!/bin/bash
# Calibrated FETCH_SIZE / WRITE_SIZE passes (tools/traffic.py) for the cfg5 and cfg2 bench lines,
# then those lines again so they carry roofline.traffic. usage: tools/gpu_traffic_cfgs.sh TAG
set -o pipefail
t=${1:-tc}
o=gpurun_out
mkdir -p $o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# streamed bytes per read: cfg5 = the first pass's bases (150) + the later passes' base image
# (2 x 38.75: 2400 B of codes + 80 B of bad bits per 64 reads); cfg2 = the bases (100)
for spec in "cfg5|k_map1 x3 passes=227.5" "cfg2|k_map1=100"; do
  c=${spec%%|*}; s=${spec#*|}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $o/${t}_${c}_$ctr -o run -- python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > $o/${t}_${c}_$ctr.log 2>&1 || { echo "$c $ctr failed"; tail -20 $o/${t}_${c}_$ctr.log; exit 1; }
  done
  python3 tools/traffic.py $c $o/${t}_${c}_FETCH_SIZE $o/${t}_${c}_WRITE_SIZE $o/${t}_traffic_$c.json "$s" > $o/${t}_traffic_$c.log 2>&1 || { echo "traffic $c failed"; cat $o/${t}_traffic_$c.log; exit 1; }
  cp $o/${t}_traffic_$c.json profiles/traffic_$c.json
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $o/${t}_bench_$c.json 2> $o/${t}_bench_$c.err || { echo "bench $c failed"; tail -20 $o/${t}_bench_$c.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$o/${t}_bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c', d['value']/1e9, d['ms_per_step'], r['frac'], r['traffic'], r.get('traffic_GBps'), (r.get('requests') or {}).get('all_per_read'))"
done
