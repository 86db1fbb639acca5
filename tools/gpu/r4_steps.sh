#!/bin/bash
# round 4: C2 step per-shape profiles: overlapped, weight gradients serial on the main stream, and main stream alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in overlap skip serial; do
  timeout -k 10 300 python -u tools/step_profile.py --tune-cache profiles/tune_r4.txt --mode $m --top 70 > gpurun_out/r4_step_$m.txt 2>&1 || { echo "FAIL $m"; tail gpurun_out/r4_step_$m.txt; exit 1; }
  head -2 gpurun_out/r4_step_$m.txt
done
