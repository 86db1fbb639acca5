#!/bin/bash
# round 5: the in_proj bias column sums inside the attention backward vs the
# separate colsum pass (ARTSBIR_ATTN_CSUM), C5 bench legs back to back
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_vit_block.py > gpurun_out/r5_csum_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r5_csum_tests.log; [ $rc = 0 ] || exit 1
B="python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2"
for v in 1 0 1; do
  ARTSBIR_ATTN_CSUM=$v timeout -k 10 600 $B > gpurun_out/r5_csum_$v.json 2>gpurun_out/r5_csum_$v.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_csum_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_csum_$v.json').read().strip().splitlines()[-1]); print('csum=$v c2', d['ms_per_step'], 'c5', d['c5']['ms_per_step'])"
done
