#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/fused.log 2>&1; rc=$?
echo "fused rc=$rc"; tail -4 gpurun_out/fused.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dgrad_bench.py > gpurun_out/dgrad_bench.txt 2>&1; rc=$?
echo "bench rc=$rc"; cat gpurun_out/dgrad_bench.txt
