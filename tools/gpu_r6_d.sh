#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r6d
mkdir -p $o
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $o/hb.log; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "repeated or multi_k" tests/test_build_gpu.py tests/test_debug_lds_gpu.py "tests/test_gpu_scale.py::test_cfg2_10k_transcripts_100bp" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { echo "tests failed"; tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in cfg2 cfg3; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-end-to-end --steps 20 > $o/b_$c.json 2> $o/b_$c.err || { echo "trace $c failed"; tail -20 $o/b_$c.err; exit 1; }
  python3 tools/bench_summary.py $o/b_$c.json | head -1
  python3 tools/trace_steps.py $o/tr_$c/run_kernel_trace.csv 2 > $o/steps_$c.txt 2>&1; head -1 $o/steps_$c.txt
done
timeout -k 10 600 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/ab/wpe5/libskq.so --config cfg5 --rounds 10 > $o/ab_wpe5_cfg5.log 2>&1 || { echo "ab failed"; tail -20 $o/ab_wpe5_cfg5.log; exit 1; }
tail -5 $o/ab_wpe5_cfg5.log
