#!/bin/bash
# (the variant this compared was removed after the run: results in profiles/r5_knn_pp.txt)
# round 5: the kNN scan with its two groups of four waves half a tile apart
# (art-sbir_amd/build_var/libpp.so, hipcc -DKNN_PP=1 on retrieval.hip: mid-tile
# barrier, group 1 one barrier behind, tile u loaded by group u & 1, 4-stage ring)
# against the production build: retrieval tests on both, then the leg base / pp / base / pp
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_retrieval_gpu.py > gpurun_out/r5_knn_pp_tests_base.log 2>&1; rc=$?
echo "tests base rc=$rc"; tail -1 gpurun_out/r5_knn_pp_tests_base.log; [ $rc = 0 ] || exit 1
ARTSBIR_LIB=$R/art-sbir_amd/build_var/libpp.so timeout -k 10 240 $T tests/test_retrieval_gpu.py > gpurun_out/r5_knn_pp_tests_pp.log 2>&1; rc=$?
echo "tests pp rc=$rc"; tail -1 gpurun_out/r5_knn_pp_tests_pp.log; [ $rc = 0 ] || exit 1
i=0
for v in base pp base pp; do
  i=$((i+1))
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libpp.so; fi
  timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r5_knn_pp_$i.log 2>&1 || { echo LEG_FAILED; tail -5 gpurun_out/r5_knn_pp_$i.log; exit 1; }
  echo "== $v"; grep noise gpurun_out/r5_knn_pp_$i.log | cut -c1-130
done
