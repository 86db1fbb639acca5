#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/pf_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/pf_tests.log
[ $rc -eq 0 ] || exit $rc
CFGS=0,1,2,3,11,12,13 timeout -k 10 300 python -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/dgrad_pf.txt; rc=$?
cat gpurun_out/dgrad_pf.txt; exit $rc
