#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5p
timeout -k 10 300 python3 tools/step_curve.py 80 > gpurun_out/r5p/curve.log 2>&1; rc=$?; tail -8 gpurun_out/r5p/curve.log; exit $rc
