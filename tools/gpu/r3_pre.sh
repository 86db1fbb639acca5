#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_preprocess_gpu.py \
  > gpurun_out/r3_pre_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|^E " gpurun_out/r3_pre_tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pre_bench.py --cpu > gpurun_out/r3_pre_bench.json 2> gpurun_out/r3_pre_bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r3_pre_bench.json; exit $rc
