#!/bin/bash
# one-wave exact merge + vectorised gallery prep: exactness tests, C4 leg, merge A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_retrieval_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_merge_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r3_merge_tests.log; exit 1; }
tail -2 gpurun_out/r3_merge_tests.log
timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r3_merge_on.log 2>&1 || { echo RETR_FAILED; tail -5 gpurun_out/r3_merge_on.log; exit 1; }
grep noise gpurun_out/r3_merge_on.log
ARTSBIR_KNN_MERGE_WAVE=0 timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r3_merge_off.log 2>&1 || { echo RETR_FAILED; tail -5 gpurun_out/r3_merge_off.log; exit 1; }
grep noise gpurun_out/r3_merge_off.log
