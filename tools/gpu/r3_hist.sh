#!/bin/bash
# kNN scan with the published-item histogram bound: exactness tests, then the C4
# leg with scan statistics, histogram on and off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_retrieval_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_hist_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r3_hist_tests.log; exit 1; }
tail -2 gpurun_out/r3_hist_tests.log
ARTSBIR_KNN_STAT=1 timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r3_hist_on.log 2>&1 || { echo RETR_FAILED; tail -5 gpurun_out/r3_hist_on.log; exit 1; }
grep noise gpurun_out/r3_hist_on.log
ARTSBIR_KNN_HIST=0 ARTSBIR_KNN_STAT=1 timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r3_hist_off.log 2>&1 || { echo RETR_FAILED; tail -5 gpurun_out/r3_hist_off.log; exit 1; }
grep noise gpurun_out/r3_hist_off.log
