#!/bin/bash
# 3x3 weight gradients of the C2 step in isolation: every candidate on the
# 56^2 x 64, 28^2 x 128, 56^2 x 128 and 112^2 stem shapes (tools/wgrad_bench.py
# SHAPES), after the halo-kernel parity tests (candidates 36-39)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py -m gpu -k "wgrad_accumulates" > gpurun_out/r4_hwg_tests.log 2>&1 || { tail -30 gpurun_out/r4_hwg_tests.log; exit 1; }
tail -1 gpurun_out/r4_hwg_tests.log
WHICH=conv SHAPES=${SHAPES:-5,6,9,10,11} timeout -k 10 400 python3 -u tools/wgrad_bench.py 2>&1 | grep -v amdgpu.ids
