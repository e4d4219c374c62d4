#!/bin/bash
# Round-4 record call: the drop-in's per-call and reference-CLI timings, smoke(), calibrated
# FETCH_SIZE / WRITE_SIZE passes (tools/traffic.py -> profiles/traffic_cfg3.json, read by the bench
# line), the default bench line (cfg3: chained tables, cpu_baseline, end-to-end leg), the kernel-
# trace stats, cfg5 / cfg2 traffic + lines (tools/gpu_traffic_cfgs.sh), a 2-rank gloo rehearsal
# of N > 1 (cpu_baseline on every rank count). The GPU test suite runs in its own call.
# usage: tools/gpu_round4.sh TAG
set -o pipefail
t=${1:-r4z}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
o=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_dropin.py tests/test_dropin_ref.py > $o/${t}_dropin.log 2>&1 || { echo "dropin failed"; tail -30 $o/${t}_dropin.log; exit 1; }
grep -E "us per|ref_cli_skq:|^skq: index" $o/${t}_dropin.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/${t}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/${t}_smoke.log; exit 1; }
echo "smoke ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $o/${t}_$c -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > $o/${t}_$c.log 2>&1 || { echo "$c failed"; tail -20 $o/${t}_$c.log; exit 1; }
done
python3 tools/traffic.py cfg3 $o/${t}_FETCH_SIZE $o/${t}_WRITE_SIZE $o/${t}_traffic_cfg3.json k_map1=150 > $o/${t}_traffic.log 2>&1 || { echo "traffic failed"; cat $o/${t}_traffic.log; exit 1; }
cp $o/${t}_traffic_cfg3.json profiles/traffic_cfg3.json
tail -5 $o/${t}_traffic.log
timeout -k 10 400 python -u bench.py > $o/${t}_bench.json 2> $o/${t}_bench.err || { echo "bench failed"; tail -20 $o/${t}_bench.err; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${t}_stats -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end > $o/${t}_stats.json 2> $o/${t}_stats.err || { echo "stats failed"; tail -20 $o/${t}_stats.err; exit 1; }
echo "stats ok"
bash tools/gpu_traffic_cfgs.sh ${t}c || { echo "cfg traffic failed"; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --reads 2000000 --steps 5 --warmup 2 > $o/${t}_bench_g2.json 2> $o/${t}_bench_g2.err || { echo "bench g2 failed"; tail -20 $o/${t}_bench_g2.err; exit 1; }
echo "bench g2 ok"
python3 - "$t" <<'PY'
import json, sys
t = sys.argv[1]
for f in ("bench", "stats", "bench_g2", "c_bench_cfg5", "c_bench_cfg2"):
    fn = "gpurun_out/%s_%s.json" % (t, f) if not f.startswith("c_") else "gpurun_out/%sc_%s.json" % (t, f[2:])
    d = json.loads(open(fn).read().strip().splitlines()[-1])
    e = d.get("end_to_end") or {}
    cb = d.get("cpu_baseline") or {}
    print(f, "value %.3f G/s" % (d["value"] / 1e9), "ms %.3f" % d["ms_per_step"], "frac %.4f" % d["roofline"]["frac"],
          "traffic", d["roofline"].get("traffic"), "e2e", e.get("reads_per_s"), "cpu", cb.get("value"), cb.get("cores"))
PY
