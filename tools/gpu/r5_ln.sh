#!/bin/bash
# round 5: the 4-column LayerNorm backward (two rows in flight per wave) against
# the 8-column form (ARTSBIR_LN_C4=0): ViT tests, then C5 bench legs back to back
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_vit_block.py tests/test_c5_gpu.py > gpurun_out/r5_ln_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r5_ln_tests.log; [ $rc = 0 ] || exit 1
B="python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2"
for v in 1 0 1; do
  ARTSBIR_LN_C4=$v timeout -k 10 600 $B > gpurun_out/r5_ln_$v.json 2>gpurun_out/r5_ln_$v.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_ln_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_ln_$v.json').read().strip().splitlines()[-1]); print('ln_c4=$v c2', d['ms_per_step'], 'c5', d['c5']['ms_per_step'])"
done
