#!/bin/bash
# round-3 closing measurement: the default bench line exactly as the driver runs
# it, then rocprofv3 kernel statistics of the C2 leg (tune cache loaded)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
s0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r3_final_bench.json 2> gpurun_out/r3_final_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r3_final_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s0 )) s"; tail -c 400 gpurun_out/r3_final_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > $R/gpurun_out/r3_prof_bench.json 2> $R/gpurun_out/r3_prof_bench.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/r3_prof_bench.err; exit 1; }
echo prof done
