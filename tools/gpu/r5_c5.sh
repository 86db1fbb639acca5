#!/bin/bash
# round 5: ViT (C5) parity tests and the C5 leg of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_c5_gpu.py tests/test_vit_block.py tests/test_losses_gpu.py > gpurun_out/r5_c5_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r5_c5_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2 > gpurun_out/r5_c5_bench.json 2>gpurun_out/r5_c5_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_c5_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r5_c5_bench.json').read().strip().splitlines()[-1]); print('c2', d['ms_per_step'], 'c5', d['c5']['ms_per_step'], d['c5']['value'])"
