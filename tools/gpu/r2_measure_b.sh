#!/bin/bash
# round 2 measurement, part B: the default bench line (CPU baselines, embed and
# retrieval legs) with the committed autotune cache, then rocprofv3 kernel
# statistics of the same command (no tuning trials in either)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
TC=$R/profiles/tune_r2.txt
timeout -k 10 700 python -u bench.py --tune-cache $TC > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
cut -c1-300 gpurun_out/bench_full.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --tune-cache $TC > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
echo done
# the C5 step (512 triplets) under the kernel trace as well
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run --output-format csv -- python3 $R/tools/c5_step.py 512 fp8 > $R/gpurun_out/c5_prof.log 2>&1 || { echo C5PROF_FAILED; tail -20 $R/gpurun_out/c5_prof.log; exit 1; }
echo c5 done
