#!/bin/bash
# ViT tests, then the weight-gradient microbenchmark (C2 conv + C5 dense shapes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/vit_tests.sh || exit $?
timeout -k 10 600 python -u tools/wgrad_bench.py > gpurun_out/wgrad_bench.txt 2>&1; rc=$?
echo "wgrad rc=$rc"; grep -v amdgpu.ids gpurun_out/wgrad_bench.txt
exit $rc
