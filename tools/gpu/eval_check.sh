#!/bin/bash
# fused inference path: encoder / C2 / CLI tests, then the embed leg of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_encoder_gpu.py tests/test_c2_gpu.py tests/test_cli_gpu.py tests/test_pgemm_gpu.py tests/test_gemm_gpu.py tests/test_modules_gpu.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/eval_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/eval_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-retrieval --no-loss-check --steps 5 --warmup 2 > gpurun_out/bench_eval.json 2> gpurun_out/bench_eval.err; rc=$?
echo "bench rc=$rc"; tail -2 gpurun_out/bench_eval.err
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_eval.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step']); print('embed', d.get('embed'))"
exit $rc
