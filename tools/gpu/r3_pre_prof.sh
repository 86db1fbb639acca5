#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/pre_prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pre_prof -o pre -- python3 tools/pre_bench.py > gpurun_out/pre_prof/out.json 2> gpurun_out/pre_prof/err.txt; rc=$?
echo "rc=$rc"; cat gpurun_out/pre_prof/out.json; find gpurun_out/pre_prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/pre_prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f"
exit $rc
