#!/bin/bash
# Record call (rounds 5-6): calibrated traffic (FETCH_SIZE / WRITE_SIZE) and instruction-count passes
# per single-GPU config, the kernel-trace stats of the default bench, then the default bench
# line itself (cfg3, with the cfg2 / cfg5 legs). The JSON the passes produce go to profiles/ on the
# box (so the bench lines read them) and to gpurun_out/ (to be committed).
# usage: tools/gpu_record.sh TAG
set -o pipefail
t=${1:-r5r}
o=gpurun_out/$t
mkdir -p $o
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $o/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# streamed bytes per read (tools/traffic.py): the bases (cfg5: the first pass's bases + the later
# passes' base image, 2 x 38.75 B)
for spec in "cfg3|k_map1=150|10000000" "cfg2|k_map1=100|1000000" "cfg5|k_map1 x3 passes=227.5|10000000"; do
  c=${spec%%|*}; rest=${spec#*|}; s=${rest%%|*}; n=${rest##*|}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $o/${c}_$ctr -o run -- python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > $o/${c}_$ctr.log 2>&1 || { echo "$c $ctr failed"; tail -20 $o/${c}_$ctr.log; exit 1; }
  done
  python3 tools/traffic.py $c $o/${c}_FETCH_SIZE $o/${c}_WRITE_SIZE $o/traffic_$c.json "$s" > $o/traffic_$c.log 2>&1 || { echo "traffic $c failed"; cat $o/traffic_$c.log; exit 1; }
  cp $o/traffic_$c.json profiles/traffic_$c.json
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $o/${c}_inst -o run -- python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > $o/${c}_inst.log 2>&1 || { echo "$c inst failed"; tail -20 $o/${c}_inst.log; exit 1; }
  python3 tools/valu_counts.py $o/${c}_inst --reads $n --config $c --probe wide --chained 1 --measured "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS over bench.py --config $c (tools/gpu_record.sh)" > $o/valu_$c.json 2> $o/valu_$c.err || { echo "valu $c failed"; cat $o/valu_$c.err; exit 1; }
  cp $o/valu_$c.json profiles/valu_$c.json
  echo "$c: traffic and instruction counts done"
done
# what binds k_map1 (cycle counters over tools/kbench.py: cfg3, 10M reads, the default chained
# tables), then the stall and LDS sets for the record
tools/pmc.sh bound $o/bound --probes auto/chain --rounds 2 > $o/bound.log 2>&1 || { echo "bound failed"; tail -20 $o/bound.log; exit 1; }
python3 tools/pmc_bound.py $o/bound k_map1 10000000 "tools/pmc.sh bound over tools/kbench.py (cfg3, 10M reads, chained), tools/pmc_bound.py; $t" > $o/pmc_bound_cfg3.json || { echo "pmc_bound failed"; exit 1; }
cp $o/pmc_bound_cfg3.json profiles/pmc_bound_cfg3.json
for set_ in stall lds; do
  tools/pmc.sh $set_ $o/$set_ --probes auto/chain --rounds 2 > $o/$set_.log 2>&1 || { echo "$set_ failed"; tail -20 $o/$set_.log; exit 1; }
done
echo "pmc sets done"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --no-extra-configs > $o/stats_bench.json 2> $o/stats_bench.err || { echo "stats bench failed"; tail -20 $o/stats_bench.err; exit 1; }
timeout -k 10 500 python3 bench.py > $o/bench.json 2> $o/bench.err || { echo "bench failed"; tail -30 $o/bench.err; exit 1; }
python3 - "$o/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("cfg3 %.3f G reads/s, %.4f ms/step, k_map1 %.4f ms, frac %.4f, bound %s, fractions %s, traffic %s" % (
    d["value"] / 1e9, d["ms_per_step"], r["avg_launch_ms"], r["frac"], r["bound"], r.get("fractions"), r.get("traffic")))
for c, x in (d.get("configs") or {}).items():
    rx = x["roofline"]
    print("%s %.3f G reads/s, %.4f ms/step, frac %.4f, bound %s, parity %s" % (c, x["value"] / 1e9, x["ms_per_step"], rx["frac"], rx["bound"], x["parity_sample"][:40]))
print("e2e", (d.get("end_to_end") or {}).get("reads_per_s"), "parity", d["parity_sample"][:40])
PY
