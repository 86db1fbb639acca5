#!/bin/bash
# round 6: the default bench line (every leg), then the rocprofv3 kernel
# statistics of the C2 leg (the line's dominant kernel must agree with it)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r6_bench.err; exit 1; }
tail -c 600 gpurun_out/r6_bench.json; echo
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r6_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6_prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 5 --warmup 2 > $R/gpurun_out/r6_prof.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/r6_prof.log; exit 1; }
find $R/gpurun_out/r6_prof -name "*kernel_stats.csv" | head -3
