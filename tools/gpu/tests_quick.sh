#!/bin/bash
# the parity tests touched this session (verbose, -s for the printed measurements)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_c2_gpu.py tests/test_encoder_gpu.py tests/test_fused_gpu.py -q -s -rf --timeout 400 --timeout-method thread -k "c2 or triplet_step or forward_branches or block_out or repack or refold" > gpurun_out/quick.log 2>&1; rc=$?
echo "quick rc=$rc"; grep -E "C2 |passed|failed|^E |FAILED" gpurun_out/quick.log | tail -30
