#!/bin/bash
# round 5: the kNN scan with four LDS stages (three tiles in flight; the slow
# path stages half a wave's rows per pass to make room), art-sbir_amd/build_var/libnst4.so
# (hipcc -DKNN_NST=4 on retrieval.hip) against the production three-stage build:
# retrieval tests on both, then the retrieval leg base / nst4 / base / nst4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_retrieval_gpu.py > gpurun_out/r5_knn_nst_tests_base.log 2>&1; rc=$?
echo "tests base rc=$rc"; tail -1 gpurun_out/r5_knn_nst_tests_base.log; [ $rc = 0 ] || exit 1
ARTSBIR_LIB=$R/art-sbir_amd/build_var/libnst4.so timeout -k 10 600 $T tests/test_retrieval_gpu.py > gpurun_out/r5_knn_nst_tests_nst4.log 2>&1; rc=$?
echo "tests nst4 rc=$rc"; tail -1 gpurun_out/r5_knn_nst_tests_nst4.log; [ $rc = 0 ] || exit 1
i=0
for v in base nst4 base nst4; do
  i=$((i+1))
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libnst4.so; fi
  timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r5_knn_nst_$i.log 2>&1 || { echo LEG_FAILED; tail -5 gpurun_out/r5_knn_nst_$i.log; exit 1; }
  echo "== $v"; grep noise gpurun_out/r5_knn_nst_$i.log | cut -c1-130
done
