#!/bin/bash
# Round-3 record call: every GPU test, smoke(), the default bench line (cfg3, with cpu_baseline and
# the end-to-end leg), cfg5 and cfg2 lines, the kernel-trace stats and FETCH_SIZE / WRITE_SIZE
# passes of the default bench (-> tools/traffic.py), and a 2-rank gloo rehearsal of N > 1.
# usage: tools/gpu_round3.sh TAG
set -o pipefail
t=${1:-r3z}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/${t}_tests.log 2>&1 || { echo "tests failed"; tail -30 $o/${t}_tests.log; exit 1; }
tail -2 $o/${t}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/${t}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/${t}_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $o/${t}_bench.json 2> $o/${t}_bench.err || { echo "bench failed"; tail -20 $o/${t}_bench.err; exit 1; }
echo "bench ok"
for c in cfg5 cfg2; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $o/${t}_bench_$c.json 2> $o/${t}_bench_$c.err || { echo "bench $c failed"; tail -20 $o/${t}_bench_$c.err; exit 1; }
done
echo "bench cfg5/cfg2 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${t}_stats -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end > $o/${t}_stats.json 2> $o/${t}_stats.err || { echo "stats failed"; tail -20 $o/${t}_stats.err; exit 1; }
echo "stats ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $o/${t}_$c -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > $o/${t}_$c.log 2>&1 || { echo "$c failed"; tail -20 $o/${t}_$c.log; exit 1; }
done
echo "pmc ok"
python3 tools/traffic.py cfg3 $o/${t}_FETCH_SIZE $o/${t}_WRITE_SIZE $o/${t}_traffic_cfg3.json k_map1=150 > $o/${t}_traffic.log 2>&1 || { echo "traffic failed"; cat $o/${t}_traffic.log; exit 1; }
cat $o/${t}_traffic.log | tail -5
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --reads 2000000 --steps 5 --warmup 2 > $o/${t}_bench_g2.json 2> $o/${t}_bench_g2.err || { echo "bench g2 failed"; tail -20 $o/${t}_bench_g2.err; exit 1; }
echo "bench g2 ok"
python3 - "$t" <<'PY'
import json, sys
t = sys.argv[1]
for f in ("bench", "bench_cfg5", "bench_cfg2", "stats", "bench_g2"):
    d = json.loads(open("gpurun_out/%s_%s.json" % (t, f)).read().strip().splitlines()[-1])
    e = d.get("end_to_end") or {}
    print(f, "value %.3f G/s" % (d["value"] / 1e9), "ms %.3f" % d["ms_per_step"], "frac %.4f" % d["roofline"]["frac"],
          "e2e", e.get("reads_per_s"), e.get("check"))
PY
