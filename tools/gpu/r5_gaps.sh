#!/bin/bash
# round 5: main-stream idle gaps and the weight-gradient tail of the C2 step,
# with and without the folded BN backward, overlapped and main stream alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fold_gpu.py > gpurun_out/r5_fold_tests.log 2>&1 || { echo FOLD_TESTS_FAILED; tail -30 gpurun_out/r5_fold_tests.log; exit 1; }
tail -1 gpurun_out/r5_fold_tests.log
for f in 1 0; do
  for m in overlap skip; do
    ARTSBIR_FOLD_BN=$f timeout -k 10 300 python -u tools/step_gaps.py --mode $m > gpurun_out/r5_gaps_f${f}_$m.txt 2>&1 || { echo FAIL $f $m; tail -20 gpurun_out/r5_gaps_f${f}_$m.txt; exit 1; }
    head -4 gpurun_out/r5_gaps_f${f}_$m.txt
  done
done
