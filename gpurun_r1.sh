#!/bin/bash
# GPU check: bench at a small batch, then full bench, then profile
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --batch 32 --steps 2 --warmup 1 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || { echo SMALL_FAILED; tail -20 gpurun_out/bench_small.err; exit 1; }
cat gpurun_out/bench_small.json | cut -c1-300
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-retrieval > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-retrieval > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
echo done
