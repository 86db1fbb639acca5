#!/bin/bash
# whole GPU suite (+ the C2 measurements printed), then the step profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x -s --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "C2 |passed|failed|^E |FAILED" gpurun_out/gpu_all.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_profile.py > gpurun_out/step_profile.txt 2>&1; rc=$?
echo "profile rc=$rc"; head -30 gpurun_out/step_profile.txt; tail -1 gpurun_out/step_profile.txt
