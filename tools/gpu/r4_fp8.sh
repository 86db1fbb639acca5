#!/bin/bash
# C5 kernels of this round: the ping-pong fp8 projection GEMM (pp8_kernel)
# against the round-3 kernel (ARTSBIR_FP8_PP=0), the one-workgroup attention
# backward and the DMA-staged forward; the ViT / C5 tests; C5 steps with the
# committed tune table
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
O=gpurun_out/r4_fp8.txt
: > $O
timeout -k 10 120 python3 tools/fp8_bench.py >> $O 2>&1 &&

timeout -k 10 120 python3 tools/attn_bench.py >> $O 2>&1 &&
ARTSBIR_ATTN_BWD2=1 timeout -k 10 120 python3 tools/attn_bench.py >> $O 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_block.py tests/test_c5_gpu.py -m gpu > gpurun_out/r4_fp8_tests.log 2>&1 &&
ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 >> $O 2>&1 &&
ARTSBIR_ATTN_BWD2=1 ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 >> $O 2>&1
rc=$?; grep -v amdgpu.ids $O; tail -3 gpurun_out/r4_fp8_tests.log; exit $rc
