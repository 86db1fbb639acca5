#!/bin/bash
# round 4: conv candidate 24 (pp64_kernel, the 512x64 ping-pong tile; measured and dropped,
# profiles/r4_pp64_ab.txt — the script needs that candidate back in the build): parity on
# every conv / dgrad / fused BN-backward case, then the conv-shape A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "-24- or 24]" -p no:cacheprovider > gpurun_out/r4_pp64_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r4_pp64_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 500 python -u tools/pp_bench.py --cands auto,22,24 --rounds 2 --only conv > gpurun_out/r4_pp64_bench.log 2>&1; rc=$?
grep -v "^round\|amdgpu.ids" gpurun_out/r4_pp64_bench.log; exit $rc
