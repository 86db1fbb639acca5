#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_retrieval_gpu.py \
  > gpurun_out/r3_retr_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r3_retr_tests.log
[ $rc -eq 0 ] || exit $rc
ARTSBIR_KNN_KB=0 timeout -k 10 300 python -u tools/retr_leg.py 2>&1 | grep noise; rc=$?
[ $rc -eq 0 ] || exit $rc
ARTSBIR_KNN_KB=1 timeout -k 10 300 python -u tools/retr_leg.py 2>&1 | grep noise
