#!/bin/bash
# round 6: the step on torch's default-priority stream (ARTSBIR_STEP_PRIO=0) vs the
# high-priority main stream (default) — C2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/r6_ab2.sh ARTSBIR_STEP_PRIO=0 && bash tools/gpu/r6_ab2.sh ARTSBIR_STEP_PRIO=0
