#!/bin/bash
# whole GPU suite, then a training-only bench line (profiled steps) and one without per-launch profiling
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-profile --steps 10 --warmup 3 > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err; rc=$?
echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_train.json
