#!/bin/bash
# round 6: shorter-lived pw256 weight-gradient workgroups beside the main stream
# (ARTSBIR_PW256_SPLITX = 2 / 4 / 16 times the split-K workgroups) — C2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for f in 4 16 2; do
  echo "== B: ARTSBIR_PW256_SPLITX=$f"
  bash tools/gpu/r6_ab2.sh ARTSBIR_PW256_SPLITX=$f || exit 1
done
