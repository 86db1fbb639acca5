#!/bin/bash
# round 6 closing run at the final commit: the GPU suite as the driver runs it,
# smoke(), the default bench line, the rocprofv3 statistics of its C2 leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/r6_suite.sh || exit 1
bash tools/gpu/r6_final.sh || exit 1
