#!/bin/bash
# round 5: the kNN scan's bound-exchange interval (KB_SYNC_TILES 64 production;
# build_var/libkb{32,128}.so) after the prefetch fix: retrieval tests on each,
# then the retrieval leg 64 / 32 / 128 / 64 / 128
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
for v in 32 128; do
  ARTSBIR_LIB=$R/art-sbir_amd/build_var/libkb$v.so timeout -k 10 300 $T tests/test_retrieval_gpu.py > gpurun_out/r5_kb_tests_$v.log 2>&1 || { echo "TESTS_FAILED $v"; tail -3 gpurun_out/r5_kb_tests_$v.log; exit 1; }
  echo "tests kb$v: $(tail -1 gpurun_out/r5_kb_tests_$v.log)"
done
i=0
for v in 64 32 128 64 128; do
  i=$((i+1))
  if [ $v = 64 ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libkb$v.so; fi
  timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r5_kb_$i.log 2>&1 || { echo LEG_FAILED; exit 1; }
  echo "== kb$v"; grep noise gpurun_out/r5_kb_$i.log | cut -c1-110
done
