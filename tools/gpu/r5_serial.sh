#!/bin/bash
# round 5: the C2 step with the weight gradients in order on the main stream
# (standalone cost of every launch) and overlapped, with and without the fold
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for f in 1 0; do
  for m in serial overlap; do
    ARTSBIR_FOLD_BN=$f timeout -k 10 300 python -u tools/step_gaps.py --mode $m --by-tag 70 > gpurun_out/r5_ser_f${f}_$m.txt 2>&1 || { echo FAIL $f $m; tail -20 gpurun_out/r5_ser_f${f}_$m.txt; exit 1; }
    head -5 gpurun_out/r5_ser_f${f}_$m.txt | tail -4
  done
done
