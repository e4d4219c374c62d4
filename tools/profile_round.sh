#!/bin/bash
# Round profile: kernel-trace stats of the default bench, then separate FETCH_SIZE / WRITE_SIZE
# passes for the roofline "traffic" field. Run on the GPU box from the repo root.
# usage: tools/profile_round.sh TAG [bench args...]   (outputs under gpurun_out/TAG_*)
set -eu
tag=$1; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
o=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${tag}_stats -o run \
  -- python3 bench.py --no-cpu-baseline --no-end-to-end "$@" > $o/${tag}_stats.json 2> $o/${tag}_stats.err
echo "stats ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $o/${tag}_$c -o run \
    -- python3 bench.py --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 "$@" > $o/${tag}_$c.log 2>&1
  echo "$c ok"
done
