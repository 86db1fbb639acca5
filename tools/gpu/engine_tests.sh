#!/bin/bash
# the engine's GPU parity tests (C2, encoder, fused batched step), then the C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_c2_gpu.py tests/test_encoder_gpu.py tests/test_fused_gpu.py tests/test_modules_gpu.py -x -q -rf --timeout 400 --timeout-method thread > gpurun_out/engine_tests.log 2>&1; rc=$?
echo "engine tests rc=$rc"; grep -E "passed|failed|^E |FAILED" gpurun_out/engine_tests.log | tail -20
exit $rc
