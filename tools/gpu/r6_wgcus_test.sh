#!/bin/bash
# round 6: the weight-gradient grids sized for fewer CUs (artsbir_set_wgrad_cus) — test
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py -k "fewer_cus" -rs \
  > gpurun_out/r6_wgcus_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r6_wgcus_tests.log; exit $rc
