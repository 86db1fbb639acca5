#!/bin/bash
# diagnosis: standalone weight-gradient candidates, then the C2 step timeline (both queues)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
WHICH=conv timeout -k 10 400 python -u tools/wgrad_bench.py > gpurun_out/wgrad_bench.txt 2>&1; rc=$?
echo "wgrad rc=$rc"; grep -v amdgpu.ids gpurun_out/wgrad_bench.txt | tail -60
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/c2_timeline.sh > /dev/null; rc=$?
echo "timeline rc=$rc"; head -40 gpurun_out/c2tl_timeline.txt
exit $rc
