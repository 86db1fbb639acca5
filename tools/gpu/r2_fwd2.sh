#!/bin/bash
# forward conv parity (segment statistics, every candidate) and microbenchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -k "fwd_segment" -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tf.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/tf.log
[ $rc -eq 0 ] || exit $rc
ONLY=0,1,2 CFGS=10 timeout -k 10 300 python -u tools/fwd_bench.py > gpurun_out/fwd2.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fwd2.txt; exit $rc
