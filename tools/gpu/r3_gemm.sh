#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CANDS=0,1,5,6,7,10,15 timeout -k 10 400 python -u tools/c2_gemm_cmp.py > gpurun_out/r3_c2_gemm_cmp2.txt 2>&1; rc=$?
echo "gemm cmp rc=$rc"; grep -v amdgpu.ids gpurun_out/r3_c2_gemm_cmp2.txt | sed -e 's/fwd_act.*hipBLASLt/| hipBLASLt/'; exit $rc
