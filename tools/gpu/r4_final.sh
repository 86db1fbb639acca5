#!/bin/bash
# round-4 final check: the GPU suite and smoke() as the driver runs them, the
# default bench line, rocprofv3 statistics of its C2 leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r4_suite.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -5 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
s0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r4_final_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s0 )) s"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4f -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > $R/gpurun_out/r4_prof_bench.json 2> $R/gpurun_out/r4_prof_bench.err || { echo PROF_FAILED; tail -5 $R/gpurun_out/r4_prof_bench.err; exit 1; }
echo prof done
