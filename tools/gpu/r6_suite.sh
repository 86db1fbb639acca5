#!/bin/bash
# round 6: the GPU suite as the driver runs it, smoke(), then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r6_suite.log; [ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/r6_suite.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -5 gpurun_out/r6_smoke.log; exit 1; }
tail -1 gpurun_out/r6_smoke.log
