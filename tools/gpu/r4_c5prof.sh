#!/bin/bash
# rocprofv3 kernel statistics of three C5 steps (ViT-B/16 fp8, 512 triplets)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ARTSBIR_TUNE_CACHE=$R/profiles/tune_r4.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run --output-format csv -- python3 $R/tools/c5_step.py 512 fp8 > $R/gpurun_out/r4_c5prof.log 2>&1
rc=$?; tail -4 $R/gpurun_out/r4_c5prof.log; exit $rc
