#!/bin/bash
# whole GPU suite and the driver's smoke() on HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_suite.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r3_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; grep -v amdgpu.ids gpurun_out/r3_smoke.log | tail -2; exit $rc
