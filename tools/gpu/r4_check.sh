#!/bin/bash
# round 4: retrieval (chunk-end bound publish), engine re-pack plan, wgrad parity after a change
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c2_gpu.py tests/test_encoder_gpu.py tests/test_fused_gpu.py tests/test_pgemm_gpu.py -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_check.log 2>&1; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/r4_check.log; exit $rc
