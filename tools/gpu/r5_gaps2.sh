#!/bin/bash
# round 5 (after the layer-1 dgrad+wgrad pass and the GLB epilogue order): the C2
# step's streams, main-stream gaps and side-stream tail, overlapped / main alone / serial
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in overlap skip serial; do
  timeout -k 10 300 python -u tools/step_gaps.py --mode $m --by-tag 40 > gpurun_out/r5_gaps2_$m.txt 2>&1 || { echo FAIL $m; tail -20 gpurun_out/r5_gaps2_$m.txt; exit 1; }
  head -5 gpurun_out/r5_gaps2_$m.txt
done
