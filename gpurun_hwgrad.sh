#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/hwgrad_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/hwgrad_tests.log; exit 1; }
tail -2 gpurun_out/hwgrad_tests.log
timeout -k 10 300 python -u scratch/wg_bench.py > gpurun_out/hwgrad_bench.txt 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/hwgrad_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/hwgrad_bench.txt
