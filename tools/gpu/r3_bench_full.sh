#!/bin/bash
# the default bench line (what the driver runs), with the tune cache written for profiling runs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --tune-cache gpurun_out/tune_r3.txt > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/r3_bench.json; exit $rc
