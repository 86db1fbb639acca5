#!/bin/bash
# GPU check: all parity tests, bench, kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-retrieval > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
echo done
