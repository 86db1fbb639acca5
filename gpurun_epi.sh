#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
SHAPES=l1_res,l1_res2t,l2_res,l3_res,l1_act1x1,l3_act3x3 CFGS=auto,0,1,3,10 timeout -k 10 300 python -u scratch/epi_bench.py > gpurun_out/epi_bench2.txt 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/epi_bench2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/epi_bench2.txt
