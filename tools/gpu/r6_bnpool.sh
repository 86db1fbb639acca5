#!/bin/bash
# round 6: the kind-1 BN-backward passes (the pooled bn2 of the strided blocks)
# read the BN input once (the ReLU mask's y_0 reused for the reduction / apply)
# against build_ab/libold.so: C2 / C1 / module tests, then C2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_c2_gpu.py tests/test_c1_gpu.py \
  tests/test_modules_gpu.py tests/test_bn_finalize_gpu.py > gpurun_out/r6_bnpool_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_bnpool_tests.log; exit 1; }
tail -2 gpurun_out/r6_bnpool_tests.log
bash tools/gpu/r6_ab2.sh ARTSBIR_LIB=$R/art-sbir_amd/build_ab/libold.so
