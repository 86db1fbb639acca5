#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_encoder_gpu.py -k "eval" \
  > gpurun_out/r3_eval_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r3_eval_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/embed_pass.py 3 --profile > gpurun_out/r3_embed_prof2.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r3_embed_prof2.txt | grep -E "profiled|res|->256 1x1|->512 1x1|->1024 1x1|->2048 1x1" | head -30; exit $rc
