#!/bin/bash
# halo-tiled conv: parity tests, then standalone timing against the other candidates
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "21 or auto" > gpurun_out/hconv_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/hconv_tests.log; exit 1; }
tail -2 gpurun_out/hconv_tests.log
SHAPES=stem3_dg,stem2_dg,l1_act3x3,stem2_fwd,stem3_fwd,l1_fwd CFGS=auto,21 timeout -k 10 300 python -u scratch/epi_bench.py > gpurun_out/hconv_bench.txt 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/hconv_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/hconv_bench.txt
