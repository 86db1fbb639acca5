#!/bin/bash
# round 5: the 64-k half-stage fp8 kernel (ARTSBIR_FP8_TILE=3)
# (the kernels this compared were removed after the run: results in profiles/r5_fp8_kloop.txt)
# against the 256 x 256 tile: parity with the tile forced, per-shape timings
# (tools/fp8_bench.py), C5 bench legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
ARTSBIR_FP8_TILE=3 timeout -k 10 600 $T tests/test_vit_block.py tests/test_c5_gpu.py > gpurun_out/r5_fp8v3_tests.log 2>&1; rc=$?
echo "tests(tile 3) rc=$rc"; tail -2 gpurun_out/r5_fp8v3_tests.log; [ $rc = 0 ] || exit 1
for t in 0 3; do
  ARTSBIR_FP8_TILE=$t timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r5_fp8v3_bench_$t.log 2>&1 || { echo FP8BENCH_FAILED; tail -5 gpurun_out/r5_fp8v3_bench_$t.log; exit 1; }
  echo "tile $t"; grep gemm gpurun_out/r5_fp8v3_bench_$t.log | cut -c1-120; grep total gpurun_out/r5_fp8v3_bench_$t.log
done
for t in 0 3; do
  ARTSBIR_FP8_NOSTORE=1 ARTSBIR_FP8_TILE=$t timeout -k 10 300 python -u tools/fp8_bench.py > gpurun_out/r5_fp8v3_ns_$t.log 2>&1 || { echo FP8BENCH_FAILED; exit 1; }
  echo "nostore tile $t"; grep total gpurun_out/r5_fp8v3_ns_$t.log
done
B="python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2"
for t in 3 0; do
  ARTSBIR_FP8_TILE=$t timeout -k 10 600 $B > gpurun_out/r5_fp8v3_$t.json 2>gpurun_out/r5_fp8v3_$t.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_fp8v3_$t.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_fp8v3_$t.json').read().strip().splitlines()[-1]); print('tile $t c5', d['c5']['ms_per_step'])"
done
