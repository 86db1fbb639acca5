#!/bin/bash
# round 5 end: rocprofv3 kernel statistics of the C2 leg (csv), then the PMC
# traffic passes of the train leg (tools/gpu/r5_pmc.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r5_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5_prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 5 --warmup 2 > $R/gpurun_out/r5_prof.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/r5_prof.log; exit 1; }
find $R/gpurun_out/r5_prof -name "*kernel_stats.csv"
cd $R && LEGS=train bash tools/gpu/r5_pmc.sh
