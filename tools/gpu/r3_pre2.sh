#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_preprocess_gpu.py \
  > gpurun_out/r3_pre_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r3_pre_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pre_bench.py > gpurun_out/r3_pre_bench.json 2> gpurun_out/r3_pre_bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r3_pre_bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/c2_gemm_cmp.py > gpurun_out/r3_c2_gemm_cmp.txt 2>&1; rc=$?
echo "gemm cmp rc=$rc"; cat gpurun_out/r3_c2_gemm_cmp.txt | grep -v amdgpu.ids; exit $rc
