#!/bin/bash
# round 4: candidate-22 parity, then re-tune every shape of every leg without the
# hipBLASLt candidate (bench.py --tune-cache none --tune-save) -> the new table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "22 or pp256" > gpurun_out/r4_t22.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r4_t22.log; [ $rc = 0 ] || exit 1
timeout -k 10 900 python -u bench.py --no-cpu-baseline --tune-cache none --tune-save gpurun_out/tune_r4.txt > gpurun_out/r4_tune_bench.json 2> gpurun_out/r4_tune_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/r4_tune_bench.json; tail -3 gpurun_out/r4_tune_bench.err; exit $rc
