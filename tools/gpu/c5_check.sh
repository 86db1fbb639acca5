#!/bin/bash
# ViT tests, then the C5 step profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu/vit_tests.sh && bash tools/gpu/c5_prof.sh > /dev/null && python3 tools/trace_steps.py gpurun_out/c5prof/run_kernel_trace.csv 2 | head -24
