#!/bin/bash
# round 6: the side (weight-gradient) stream on all but a few CUs (ARTSBIR_SIDE_CUS
# = 248 / 240 / 224 of 256, spread over the XCDs), so the main stream's small
# kernels always find a CU the side stream's long-lived workgroups do not hold — C2 A/B
# (second run: the weight-gradient grids sized for those CUs, artsbir_set_wgrad_cus)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for f in ${SIDE_LIST:-248 240 224}; do
  echo "== B: ARTSBIR_SIDE_CUS=$f"
  bash tools/gpu/r6_ab2.sh ARTSBIR_SIDE_CUS=$f || exit 1
done
