#!/bin/bash
# kernel microbenchmarks: BN-backward apply / forward / fused dgrad shapes, then the step profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py tests/test_c2_gpu.py tests/test_fused_gpu.py -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/kb_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/kb_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fwd_bench.py > gpurun_out/fwd_bench.txt 2>&1; rc=$?
echo "fwd rc=$rc"; grep -v amdgpu.ids gpurun_out/fwd_bench.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_profile.py --mode skip > gpurun_out/step_profile_skip.txt 2>&1; rc=$?
echo "profile rc=$rc"; head -3 gpurun_out/step_profile_skip.txt; grep "bn_bwd_apply" gpurun_out/step_profile_skip.txt | head; tail -1 gpurun_out/step_profile_skip.txt
