#!/bin/bash
# whole GPU suite, the default bench line (tune cache loaded), C5 under the kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --tune-cache $R/profiles/tune_r2.txt > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
cut -c1-200 gpurun_out/bench_full.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run --output-format csv -- python3 $R/tools/c5_step.py 512 fp8 > $R/gpurun_out/c5_prof.log 2>&1 || { echo C5PROF_FAILED; tail -20 $R/gpurun_out/c5_prof.log; exit 1; }
grep step $R/gpurun_out/c5_prof.log
