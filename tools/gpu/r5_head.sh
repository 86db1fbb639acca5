#!/bin/bash
# round 5: the attention-pool weight gradients on the side stream: parity tests, C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_c2_gpu.py tests/test_c1_gpu.py tests/test_modules_gpu.py tests/test_encoder_gpu.py tests/test_ddp_gpu.py tests/test_fused_gpu.py::test_forward_branches_matches_separate_calls > gpurun_out/r5_head_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r5_head_tests.log; [ $rc = 0 ] || exit 1
B="python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 10 --warmup 3"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/r5_head_$i.json 2>/dev/null || { echo BENCH_FAILED; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_head_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['streams_kernel_ms'])"
done
