#!/bin/bash
# round 4: the whole GPU suite (as the driver runs it) + smoke
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/r4_suite.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1; rc=$?
cat gpurun_out/r4_smoke.log | tail -2; exit $rc
