#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vit_block.py -v -s -rf --timeout 200 --timeout-method thread > gpurun_out/vit_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert|passed|failed|mismatch" gpurun_out/vit_tests.log | tail -30
exit $rc
