#!/bin/bash
# round 6: one persistent halo weight-gradient workgroup per CU instead of two
# (ARTSBIR_HWGRAD_PERCU=1), so the main stream's kernels fit beside it — C2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/r6_ab2.sh ARTSBIR_HWGRAD_PERCU=1
