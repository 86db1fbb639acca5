#!/bin/bash
# full bench line (no CPU baseline) + rocprofv3 kernel trace of the same command
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_quick.json 2> $R/gpurun_out/bench_quick.err || { echo BENCH_FAILED; tail -20 $R/gpurun_out/bench_quick.err; exit 1; }
cut -c1-400 $R/gpurun_out/bench_quick.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_quick -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-retrieval > $R/gpurun_out/bench_quick_prof.json 2> $R/gpurun_out/bench_quick_prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_quick_prof.err; exit 1; }
echo done
