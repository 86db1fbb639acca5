#!/bin/bash
# round 6: the streaming RES data gradient (candidate 26, csrc/rstream.hip):
# fused-dgrad tests with it forced, then its time against the tuned kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -x -q -rs -k "dgrad_fused and (26 or auto)" --timeout 300 --timeout-method thread > gpurun_out/r6_rstream_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r6_rstream_tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6_rstream_tests.log | head -20; exit 1; }
CFGS=18,16,22,26 SHAPES=4,6,7 timeout -k 10 300 python -u tools/dgrad_bench.py > gpurun_out/r6_rstream_bench.txt 2>&1; rc=$?
cat gpurun_out/r6_rstream_bench.txt; exit $rc
