#!/bin/bash
# 32-k-stage persistent forward candidate (cfg 15): parity, forward microbenchmark, C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tps32.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/tps32.log
[ $rc -eq 0 ] || exit $rc
CFGS=10,15 timeout -k 10 300 python -u tools/fwd_bench.py 2>&1 | grep -v amdgpu.ids | grep -E "==|stats1"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-c5 --no-profile --steps 10 --warmup 3 > gpurun_out/bps32.json 2> gpurun_out/bps32.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bps32.json'));print(d['ms_per_step'],d['value'], d['embed']['value'])"
exit $rc
