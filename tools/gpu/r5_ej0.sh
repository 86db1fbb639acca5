#!/bin/bash
# (the variant this compared was the committed one: the change was reverted after the run, results in profiles/r5_pp256_ej0.txt)
# round 5: pp256's epilogue operand batch for BK 0 (residual / QuickGELU gate):
# all 8 pixel tiles of a channel pair at once (production) against 4
# (art-sbir_amd/build_var/libej4.so, -DPP_EJB0=4): pp256 / ViT tests, the gate
# GEMM alone (tools/gate_bench.py), then the bench's C2 + C5 legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_pgemm_gpu.py tests/test_vit_block.py tests/test_c5_gpu.py > gpurun_out/r5_ej0_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/r5_ej0_tests.log; [ $rc = 0 ] || exit 1
for v in base ej4; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libej4.so; fi
  ARTSBIR_TUNE_CACHE=$R/profiles/tune_r5.txt timeout -k 10 300 python -u tools/gate_bench.py > gpurun_out/r5_ej0_gate_$v.log 2>&1 || { echo FAILED; exit 1; }
  echo "== $v"; grep run gpurun_out/r5_ej0_gate_$v.log
done
B="python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2"
i=0
for v in base ej4 base ej4; do
  i=$((i+1))
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libej4.so; fi
  timeout -k 10 600 $B > gpurun_out/r5_ej0_$i.json 2>gpurun_out/r5_ej0_$i.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_ej0_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_ej0_$i.json').read().strip().splitlines()[-1]); print('$v c2', d['ms_per_step'], 'c5', d['c5']['ms_per_step'])"
done
