#!/bin/bash
# round 4: the ping-pong 256x256 tile (candidates 22 / 23): kernel parity against
# torch on every conv / dgrad / fused BN-backward case, then the shape A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "-22- or -23- or 22] or 23]" > gpurun_out/r4_pp_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r4_pp_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 500 python -u tools/pp_bench.py --cands ${CANDS:-0,5,19,22} --rounds 2 > gpurun_out/r4_pp_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r4_pp_bench.log | grep -v "round"; exit $rc
