#!/bin/bash
# round 5: the kNN scan's chunk length balanced to the CU count (ARTSBIR_KNN_BALANCE,
# C4: 32 chunks of 245 tiles instead of 31 of 256): retrieval tests, then the
# retrieval leg (tools/retr_leg.py) with balancing on / off / on
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_retrieval_gpu.py > gpurun_out/r5_knn_bal_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r5_knn_bal_tests.log; [ $rc = 0 ] || exit 1
for v in 1 0 1; do
  ARTSBIR_KNN_BALANCE=$v timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r5_knn_bal_$v.log 2>&1 || { echo LEG_FAILED; tail -5 gpurun_out/r5_knn_bal_$v.log; exit 1; }
  echo "balance=$v"; grep noise gpurun_out/r5_knn_bal_$v.log | cut -c1-160
done
