#!/bin/bash
# kernel statistics of the C4 retrieval leg (rocprofv3 --kernel-trace --stats)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_retr -o run --output-format csv -- python3 $R/tools/retr_leg.py > $R/gpurun_out/retr_prof.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/retr_prof.log; exit 1; }
grep noise $R/gpurun_out/retr_prof.log
head -20 $R/gpurun_out/prof_retr/run_kernel_stats.csv | cut -c1-200
