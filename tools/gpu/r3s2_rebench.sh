#!/bin/bash
# round-3 session-2 closing bench at the final commit: the default bench line and
# rocprofv3 kernel statistics of its C2 leg (traffic files from r3s2_closing.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
s0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r3s2_final_bench.json 2> gpurun_out/r3s2_final_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r3s2_final_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s0 )) s"; tail -c 200 gpurun_out/r3s2_final_bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_r3s2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3s2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > $R/gpurun_out/r3s2_prof_bench.json 2> $R/gpurun_out/r3s2_prof_bench.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/r3s2_prof_bench.err; exit 1; }
echo prof done
