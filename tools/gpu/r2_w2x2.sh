#!/bin/bash
# candidate 5 (256x256 tile, 4 waves of 128x128): parity tests, forward / dgrad microbenchmarks, C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t5.log
[ $rc -eq 0 ] || exit $rc
ONLY=5,6,7,8 CFGS=0,5,10 timeout -k 10 300 python -u tools/fwd_bench.py > gpurun_out/fwd5.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fwd5.txt
[ $rc -eq 0 ] || exit $rc
CFGS=0,3,5 timeout -k 10 300 python -u tools/dgrad_bench.py > gpurun_out/dgrad5.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dgrad5.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --steps 10 --warmup 3 > gpurun_out/b5.json 2> gpurun_out/b5.err; rc=$?
echo "bench rc=$rc"; python3 -c "
import json;d=json.load(open('gpurun_out/b5.json'));print(d['ms_per_step'],d['value']);r=d['roofline'];print(r['kernel'],r['frac']);
[print(k,v) for k,v in list(r['per_kernel'].items())[:16]]"
exit $rc
