#!/bin/bash
# fused / plain data-gradient microbenchmark over every tile configuration
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CFGS=${CFGS:-0,1,2,3,10} timeout -k 10 300 python -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/dgrad_all.txt
