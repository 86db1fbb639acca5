#!/bin/bash
# round 6: the kNN scan with 64 queries per wave (4 waves, one per SIMD, both
# halves' A fragments resident: ARTSBIR_KNN_QH=2) against 32 (8 waves): the
# retrieval / fp32-order tests on both, then the leg qh1 / qh2 / qh1 / qh2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
ARTSBIR_KNN_QH=2 timeout -k 10 400 $T tests/test_retrieval_gpu.py tests/test_fp32_order.py > gpurun_out/r6_knn_qh_tests2.log 2>&1; rc=$?
echo "tests qh2 rc=$rc"; tail -1 gpurun_out/r6_knn_qh_tests2.log; [ $rc = 0 ] || { tail -30 gpurun_out/r6_knn_qh_tests2.log; exit 1; }
i=0
for v in 1 2 1 2; do
  i=$((i+1))
  ARTSBIR_KNN_QH=$v timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r6_knn_qh_$i.log 2>&1 || { echo LEG_FAILED; tail -5 gpurun_out/r6_knn_qh_$i.log; exit 1; }
  echo "== qh$v"; grep -v amdgpu.ids gpurun_out/r6_knn_qh_$i.log | cut -c1-160 | tail -4
done
