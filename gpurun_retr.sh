#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_retrieval_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/retr_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/retr_tests.log; exit 1; }
tail -1 gpurun_out/retr_tests.log
timeout -k 10 300 python -u scratch/retr_bench.py > gpurun_out/retr_bench.json 2> gpurun_out/retr_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/retr_bench.err; exit 1; }
cat gpurun_out/retr_bench.json
