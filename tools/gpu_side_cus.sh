set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r6y; mkdir -p $o
for v in 0 64 128 32 0; do
  if [ $v = 0 ]; then unset SKQ_DEV SKQ_SIDE_CUS; else export SKQ_DEV=1 SKQ_SIDE_CUS=$v; fi
  timeout -k 10 200 python3 bench.py --config cfg3 --no-cpu-baseline --no-end-to-end > $o/cus_$v.json 2> $o/cus_$v.err || { echo "cus $v failed"; tail -5 $o/cus_$v.err; exit 1; }
  echo -n "side CUs $v: "; python3 tools/bench_summary.py $o/cus_$v.json | head -1
done
