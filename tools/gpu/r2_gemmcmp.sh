#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_lib_cmp.py > gpurun_out/gemmcmp.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/gemmcmp.txt; exit $rc
