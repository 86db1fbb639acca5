#!/bin/bash
# retrieval kernels: parity tests, then the 1M x 512 leg per scan kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_retrieval_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/retr_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/retr_tests.log; exit 1; }
tail -3 gpurun_out/retr_tests.log
timeout -k 10 300 python -u tools/retr_bench.py auto auto-noshare > gpurun_out/retr_bench.json 2> gpurun_out/retr_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/retr_bench.err; exit 1; }
cut -c1-700 gpurun_out/retr_bench.json
