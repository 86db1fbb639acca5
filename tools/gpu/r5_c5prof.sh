#!/bin/bash
# round 5: every kernel of the C5 (ViT-B/16 fp8, 512 triplets) step under
# rocprofv3 --stats (the bench line's per_kernel covers the GEMM / attention calls only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r5_c5prof
ARTSBIR_TUNE_CACHE=$R/profiles/tune_r5.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5_c5prof -o run -- python3 $R/tools/c5_step.py 512 fp8 > $R/gpurun_out/r5_c5prof.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/r5_c5prof.log; exit 1; }
grep -v "^W2\|^E2" $R/gpurun_out/r5_c5prof.log | tail -5
head -40 $R/gpurun_out/r5_c5prof/run_kernel_stats.csv | cut -c1-200
