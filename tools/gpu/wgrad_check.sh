#!/bin/bash
# wgrad correctness over all candidates, then the microbenchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pgemm_gpu.py -q -x -k "wgrad or gemm_tn" --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/wgrad_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/wgrad_bench.py > gpurun_out/wgrad_bench.txt 2>&1; rc=$?
echo "wgrad rc=$rc"; grep -v amdgpu.ids gpurun_out/wgrad_bench.txt
exit $rc
