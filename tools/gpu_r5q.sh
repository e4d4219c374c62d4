#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5q
mkdir -p $O
for a in "" "--no-settle" ""; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 $a > $O/b.log 2> $O/b.err || { echo "bench rc=$?"; tail $O/b.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b.log').read().strip().splitlines()[-1])
r=d['roofline']
print('$a', '%.3f G/s %.4f ms/step settle %s k_map1 %.4f frac %.4f valu %.4f bound %s' % (d['value']/1e9, d['ms_per_step'], d.get('settle_steps'), r['avg_launch_ms'], r['frac'], (r.get('valu') or {}).get('frac', 0), r['bound']))
for c, x in (d.get('configs') or {}).items():
    print('  ', c, '%.3f G/s %.4f ms/step settle %s frac %.4f' % (x['value']/1e9, x['ms_per_step'], x.get('settle_steps'), x['roofline']['frac']))
print('  e2e', d['end_to_end']['reads_per_s'], d['parity_sample'][:30])"
  cp $O/b.log $O/b_last.json
done
