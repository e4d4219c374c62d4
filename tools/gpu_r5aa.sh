#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5aa
timeout -k 10 400 python3 tools/abbench.py sketch-for-rna-seq_amd/lib/libskq.so --config cfg5 --rounds 12 --env-b SKQ_DEV=1,SKQ_ABLATE=64 > gpurun_out/r5aa/ab.log 2>&1; rc=$?
tail -4 gpurun_out/r5aa/ab.log
[ $rc -eq 0 ] || [ $rc -eq 2 ]
