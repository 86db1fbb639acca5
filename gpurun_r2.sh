#!/bin/bash
# kernel tests for the conv paths, then the per-shape step profile
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 || { echo FUSED_TESTS_FAILED; tail -40 gpurun_out/fused_tests.log; exit 1; }
tail -2 gpurun_out/fused_tests.log
timeout -k 10 300 python scratch/shape_profile.py > gpurun_out/shape_profile.txt 2>&1 || { echo PROFILE_FAILED; tail -20 gpurun_out/shape_profile.txt; exit 1; }
head -45 gpurun_out/shape_profile.txt
