#!/bin/bash
# the tests added this round (DDP overlap on the engine, CLI second pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_preprocess_gpu.py tests/test_modules_gpu.py tests/test_ddp_gpu.py tests/test_cli_gpu.py -x -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|rank |passed|failed" gpurun_out/new_tests.log | tail -20
exit $rc
