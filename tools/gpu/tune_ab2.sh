#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --steps 3 --warmup 2"
timeout -k 10 300 $B --tune-cache gpurun_out/tune_fresh.txt > gpurun_out/ab2_notune.json 2>/dev/null || exit 1
timeout -k 10 300 $B --tune-cache profiles/tune_r2.txt > gpurun_out/ab2_cache.json 2>/dev/null || exit 1
echo ok
