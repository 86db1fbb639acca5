#!/bin/bash
# round 6: split-K form of the fold's small GEMMs (fold_gemm_kernel) — tests,
# standalone times at the C2 shapes against the unsplit build, C2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OLD=$R/art-sbir_amd/build_ab/libartsbir_nosplit.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fold_gpu.py \
  -k "prep or combine or toggles or offset" > gpurun_out/r6_foldsplit_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_foldsplit_tests.log; exit 1; }
tail -2 gpurun_out/r6_foldsplit_tests.log
echo "== split" > gpurun_out/r6_foldsplit_bench.txt
timeout -k 10 120 python -u tools/fold_gemm_bench.py >> gpurun_out/r6_foldsplit_bench.txt 2>&1 || exit 1
echo "== nosplit" >> gpurun_out/r6_foldsplit_bench.txt
ARTSBIR_LIB=$OLD timeout -k 10 120 python -u tools/fold_gemm_bench.py >> gpurun_out/r6_foldsplit_bench.txt 2>&1 || exit 1
cat gpurun_out/r6_foldsplit_bench.txt
bash tools/gpu/r6_ab2.sh ARTSBIR_LIB=$OLD
