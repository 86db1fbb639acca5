#!/bin/bash
# 32-k-stage 256x256 candidate (cfg 5): parity, microbenchmarks, C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tk32.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/tk32.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/gemm_lib_cmp.py 2>&1 | grep -v amdgpu.ids | grep NT
ONLY=0,1,2,3,6,7,8 CFGS=0,5 timeout -k 10 300 python -u tools/fwd_bench.py 2>&1 | grep -v amdgpu.ids | grep -E "==|stats1"
CFGS=0,3,5 timeout -k 10 300 python -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 10 --warmup 3 > gpurun_out/bk32.json 2> gpurun_out/bk32.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bk32.json'));print(d['ms_per_step'],d['value'])"
exit $rc
