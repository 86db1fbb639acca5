#!/bin/bash
# per-launch profile of the C2 step, the attention-pool GEMM rows
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_profile.py --steps 2 --mode skip --top 200 > gpurun_out/sp.txt 2>&1; rc=$?
grep -E "gemm_|conv_gemm|attn" gpurun_out/sp.txt | head -30; exit $rc
