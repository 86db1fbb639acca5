#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5prof -o run --output-format csv -- python3 $R/tools/c5_step.py 128 fp8 > $R/gpurun_out/c5_step.log 2>&1; rc=$?
echo "rc=$rc"; grep step $R/gpurun_out/c5_step.log
f=$(find $R/gpurun_out/c5prof -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -c1-220
