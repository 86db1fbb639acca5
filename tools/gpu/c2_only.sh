#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_c2_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/c2.log 2>&1; rc=$?
echo "c2 rc=$rc"; grep -E "PASS|FAIL|ERROR|C2 bf16|passed|failed|^E " gpurun_out/c2.log | tail -30
