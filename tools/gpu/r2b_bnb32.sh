#!/bin/bash
# candidate 16 (persistent fused BN-backward dgrad, 32-k stages): parity, dgrad microbenchmark, C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t16.log
[ $rc -eq 0 ] || exit $rc
CFGS=0,3,14,16 timeout -k 10 300 python -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids | grep -E "==|bnb"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 10 --warmup 3 > gpurun_out/b16.json 2> gpurun_out/b16.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/b16.json'));print(d['ms_per_step'],d['value'])"
exit $rc
