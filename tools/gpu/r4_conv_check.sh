#!/bin/bash
# parity of every conv / GEMM kernel family after an epilogue change, then the C2 leg
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py tests/test_c2_gpu.py tests/test_c1_gpu.py tests/test_encoder_gpu.py tests/test_gemm_gpu.py -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_conv_check.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r4_conv_check.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 10 --warmup 3 > gpurun_out/r4_conv_check.json 2> gpurun_out/r4_conv_check.err || { tail -5 gpurun_out/r4_conv_check.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4_conv_check.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'], d.get('loss_step0_rel_diff'))"
