#!/bin/bash
# session-2 baseline: quick parity tests, C2 bench leg, then standalone weight-gradient shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/tests_quick.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_base.json 2> gpurun_out/s2_base.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_base.err; exit 1; }
tail -c 600 gpurun_out/s2_base.json
timeout -k 10 400 python -u tools/wgrad_bench.py > gpurun_out/s2_wgrad_bench.txt 2>&1 || { echo WG_FAILED; tail -20 gpurun_out/s2_wgrad_bench.txt; exit 1; }
grep '==' gpurun_out/s2_wgrad_bench.txt
