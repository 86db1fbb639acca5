#!/bin/bash
# per-kernel breakdown of one C5 step at the bench batch (512 triplets)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/c5bd -o run --output-format csv -- python3 $R/tools/c5_step.py ${C5B:-512} fp8 > $R/gpurun_out/c5bd.log 2>&1 || exit $?
f=$(find $R/gpurun_out/c5bd -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_steps.py "$f" 2 > $R/gpurun_out/c5_breakdown.txt && head -32 $R/gpurun_out/c5_breakdown.txt
rm -f "$f"
