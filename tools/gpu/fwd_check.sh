#!/bin/bash
# encoder / fused / gemm tests, then the forward-conv microbenchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py tests/test_c2_gpu.py tests/test_fused_gpu.py tests/test_gemm_gpu.py tests/test_pgemm_gpu.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/fc_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/fc_tests.log
[ $rc -eq 0 ] || exit $rc
CFGS=${CFGS:-0,10} timeout -k 10 300 python -u tools/fwd_bench.py > gpurun_out/fwd_bench.txt 2>&1; rc=$?
echo "fwd rc=$rc"; grep -v amdgpu.ids gpurun_out/fwd_bench.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_profile.py --mode skip > gpurun_out/step_profile_skip.txt 2>&1; rc=$?
echo "profile rc=$rc"; head -2 gpurun_out/step_profile_skip.txt; tail -1 gpurun_out/step_profile_skip.txt
