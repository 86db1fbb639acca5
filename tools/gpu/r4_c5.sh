#!/bin/bash
# C5 change check: the ViT / C5 GPU tests, three C5 steps (tune_r4.txt), then
# rocprofv3 kernel statistics of the same steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_block.py tests/test_c5_gpu.py -m gpu > gpurun_out/r4_c5_tests.log 2>&1 || { tail -30 gpurun_out/r4_c5_tests.log; exit 1; }
tail -2 gpurun_out/r4_c5_tests.log
ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
ARTSBIR_TUNE_CACHE=$R/profiles/tune_r4.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run --output-format csv -- python3 $R/tools/c5_step.py 512 fp8 > $R/gpurun_out/r4_c5prof.log 2>&1 || { tail -5 $R/gpurun_out/r4_c5prof.log; exit 1; }
echo prof ok
