#!/bin/bash
# round 5: the kNN scan's B-fragment prefetch depth 4 (no spill; production)
# against 6 (a 16-B spill reloaded behind s_waitcnt vmcnt(0) every tile;
# art-sbir_amd/build_var/libpf6.so built with -DKNN_PF=6): retrieval tests on the
# production build, then the retrieval leg (tools/retr_leg.py) base / pf6 / base
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_retrieval_gpu.py > gpurun_out/r5_knn_pf_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r5_knn_pf_tests.log; [ $rc = 0 ] || exit 1
i=0
for v in base pf6 base; do
  i=$((i+1))
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libpf6.so; fi
  timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r5_knn_pf_$i.log 2>&1 || { echo LEG_FAILED; tail -5 gpurun_out/r5_knn_pf_$i.log; exit 1; }
  echo "== $v"; grep noise gpurun_out/r5_knn_pf_$i.log | cut -c1-130
done
