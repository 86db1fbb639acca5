#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_encoder_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bits_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/bits_tests.log; exit 1; }
tail -1 gpurun_out/bits_tests.log
bash gpurun_env.sh bits1:ARTSBIR_STEP_PRIO=-1 bits0:ARTSBIR_MASK_BITS=0,ARTSBIR_STEP_PRIO=-1 bits1b:ARTSBIR_STEP_PRIO=-1 bits0b:ARTSBIR_MASK_BITS=0,ARTSBIR_STEP_PRIO=-1
