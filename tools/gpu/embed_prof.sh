#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/embprof -o run --output-format csv -- python3 $R/tools/embed_pass.py 12 > $R/gpurun_out/embprof.log 2>&1; rc=$?
echo "rc=$rc"
f=$(find $R/gpurun_out/embprof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_window.py "$f" 12
