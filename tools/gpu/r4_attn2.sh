#!/bin/bash
# attention epilogue with 16-B stores (v_permlane32_swap): ViT/C5 tests, attention timing, C5 steps
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_block.py tests/test_c5_gpu.py -m gpu -p no:cacheprovider > gpurun_out/r4_attn2_tests.log 2>&1 || { tail -30 gpurun_out/r4_attn2_tests.log; exit 1; }
tail -1 gpurun_out/r4_attn2_tests.log
timeout -k 10 120 python3 tools/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 2>&1 | grep -v amdgpu.ids
