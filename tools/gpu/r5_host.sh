#!/bin/bash
# round 5: is the host ever behind the GPU in the C2 step?  Host issue time vs
# GPU start of every main-stream launch, for a step issued right after a sync
# and for one issued while the GPU still runs the previous step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for pre in 0 1; do
  timeout -k 10 300 python -u tools/step_gaps.py --mode overlap --host --pre $pre > gpurun_out/r5_host_pre$pre.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/r5_host_pre$pre.txt; exit 1; }
  grep -A25 "started within" gpurun_out/r5_host_pre$pre.txt | head -30
done
