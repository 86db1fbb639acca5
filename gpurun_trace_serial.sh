#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARTSBIR_OVERLAP_WGRAD=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serial -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-retrieval --no-profile > $R/gpurun_out/bench_serial.json 2> $R/gpurun_out/bench_serial.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/bench_serial.err; exit 1; }
echo done
