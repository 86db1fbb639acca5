#!/bin/bash
# 3x3 weight gradients of the C2 step in isolation: every candidate on the
# 56^2 x 64, 28^2 x 128 and 56^2 x 128 shapes (tools/wgrad_bench.py SHAPES)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
WHICH=conv SHAPES=${SHAPES:-5,6,9} timeout -k 10 300 python3 -u tools/wgrad_bench.py 2>&1 | grep -v amdgpu.ids
