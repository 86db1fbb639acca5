#!/bin/bash
# kernel trace of a short C2 bench run and the last step's timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c2tl -o run -- python3 bench.py --steps 3 \
  --warmup 3 --no-c5 --no-embed --no-retrieval --no-cpu-baseline --no-loss-check --no-profile > gpurun_out/c2tl.log 2>&1 || exit $?
f=$(find gpurun_out/c2tl -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/c2tl_timeline.txt && cat gpurun_out/c2tl_timeline.txt
rm -f "$f"
