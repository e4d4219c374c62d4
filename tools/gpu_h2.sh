mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-end-to-end > gpurun_out/h2_cfg5_stash.json 2> gpurun_out/h2_cfg5_stash.err || exit 1
SKQ_STASH=0 timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-end-to-end > gpurun_out/h2_cfg5_nostash.json 2> gpurun_out/h2_cfg5_nostash.err || exit 1
timeout -k 10 200 python -u bench.py --config cfg5 --no-cpu-baseline --no-end-to-end > gpurun_out/h2_cfg5_stash2.json 2> gpurun_out/h2_cfg5_stash2.err || exit 1
for f in h2_cfg5_stash h2_cfg5_nostash h2_cfg5_stash2; do python -c "import json,sys;d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]);print('$f',d['value']/1e9,d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d.get('parity_sample'))"; done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/h2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/h2_tests.log; exit $rc
