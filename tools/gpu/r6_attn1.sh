#!/bin/bash
# round 6: attention backward with P / dS computed once per tile (attn_bwd1_kernel)
# — tests, attn_bench A/B against the two-sided form (ARTSBIR_ATTN_BWD1=0), C5 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vit_block.py tests/test_c5_gpu.py \
  > gpurun_out/r6_attn1_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_attn1_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn1_tests.log
for i in 1 2; do
  echo -n "new "; timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep bwd || exit 1
  echo -n "old "; ARTSBIR_ATTN_BWD1=0 timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep bwd || exit 1
done
C5="--no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-loss-check --no-profile --steps 5 --warmup 2"
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then E="ARTSBIR_ATTN_BWD1=0"; else E=""; fi
    env $E timeout -k 10 300 python -u bench.py $C5 > gpurun_out/r6_attn1_$v.log 2>&1 || { echo RUN_FAILED; tail -5 gpurun_out/r6_attn1_$v.log; exit 1; }
    tail -1 gpurun_out/r6_attn1_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'C2', d['ms_per_step'], 'C5', d['c5']['ms_per_step'], d['c5']['value'])"
  done
done
