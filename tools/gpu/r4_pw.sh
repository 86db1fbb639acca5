#!/bin/bash
# round 4: pw256 wgrad parity + A/B on the C2 / C5 weight-gradient shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "pw256" > gpurun_out/r4_pw_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/r4_pw_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u tools/wg_bench.py > gpurun_out/r4_wg_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -v "^round" gpurun_out/r4_wg_bench.log; exit $rc
