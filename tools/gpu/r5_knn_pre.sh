#!/bin/bash
# (the variant this compared was reverted after the run: results in profiles/r5_knn_pre.txt)
# round 5: the kNN prefilter ahead of the per-tile barrier (production, KNN_PRE=1)
# against after it (build_var/libpre0.so): retrieval tests, then the leg
# pre / post / pre / post
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_retrieval_gpu.py > gpurun_out/r5_pre_tests.log 2>&1 || { echo TESTS_FAILED; tail -3 gpurun_out/r5_pre_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r5_pre_tests.log)"
i=0
for v in pre post pre post; do
  i=$((i+1))
  if [ $v = pre ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libpre0.so; fi
  timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r5_pre_$i.log 2>&1 || { echo LEG_FAILED; exit 1; }
  echo "== $v"; grep noise gpurun_out/r5_pre_$i.log | cut -c1-110
done
