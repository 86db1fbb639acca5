#!/bin/bash
# round 4: pp256 K-tile segment shares (diagnostic stamp build), then the new C1 parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python -u tools/pp_stamp.py 302592 768 2304 > gpurun_out/r4_stamp.log 2>&1; rc=$?
cat gpurun_out/r4_stamp.log; [ $rc = 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_c1_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r4_c1.log 2>&1; rc=$?
tail -30 gpurun_out/r4_c1.log; exit $rc
