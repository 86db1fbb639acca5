#!/bin/bash
# round 6: attn_bwd1_kernel (slot phases) — tests and attn_bench A/B only
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vit_block.py \
  > gpurun_out/r6_attn1b_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_attn1b_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn1b_tests.log
for i in 1 2; do
  echo -n "new "; timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep bwd || exit 1
  echo -n "old "; ARTSBIR_ATTN_BWD1=0 timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep bwd || exit 1
done
