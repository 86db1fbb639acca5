#!/bin/bash
# fp8 GEMM: 256x128 3-stage tile vs the 256x256 2-stage tile (parity tests, then the C5 shapes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vit_block.py tests/test_c5_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_fp8_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r3_fp8_tests.log; exit 1; }
tail -1 gpurun_out/r3_fp8_tests.log
for bn in 128 256; do
  for ns in 0 1; do
    ARTSBIR_FP8_BN=$bn ARTSBIR_FP8_NOSTORE=$ns timeout -k 10 200 python -u tools/fp8_bench.py > gpurun_out/r3_fp8_bn${bn}_ns$ns.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r3_fp8_bn${bn}_ns$ns.log; exit 1; }
    echo "bn=$bn nostore=$ns"; grep gemm gpurun_out/r3_fp8_bn${bn}_ns$ns.log | cut -c1-120
  done
done
