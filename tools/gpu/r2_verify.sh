#!/bin/bash
# round-2 re-entry check: whole GPU suite, default bench line, rocprofv3 stats of the training leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; rc=$?
echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_full.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --steps 5 --warmup 2 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err; rc=$?
echo "prof rc=$rc"; exit $rc
