#!/bin/bash
# round 6 (final kernels): bench.py --gpus 2 rehearsed on one GPU over gloo
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ARTSBIR_DIST_BACKEND=gloo timeout -k 10 800 python -u bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r6_gloo2b.log 2>&1; rc=$?
tail -c 1200 gpurun_out/r6_gloo2b.log; exit $rc
