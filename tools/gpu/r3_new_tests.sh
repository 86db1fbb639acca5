#!/bin/bash
# round 3: the new GPU tests (C5 full size, 2-rank train.main, eval refold), then a C5-only bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_c5_gpu.py tests/test_train_ddp_gpu.py \
  "tests/test_encoder_gpu.py::test_fused_eval_refolds_after_train_forward_without_step" \
  > gpurun_out/r3_new_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|C5 |step-0" gpurun_out/r3_new_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --no-retrieval --no-embed --no-cpu-baseline \
  > gpurun_out/r3_bench_c5.json 2> gpurun_out/r3_bench_c5.err; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/r3_bench_c5.json; exit $rc
