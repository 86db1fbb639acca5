#!/bin/bash
# round-3 session-2: the GPU test suite (as the driver runs it) and smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r3s2_gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r3s2_gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s2_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r3s2_smoke.log; exit $rc
