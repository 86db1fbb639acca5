#!/bin/bash
# (the change this compared was reverted after the run: results appended to profiles/r5_pp256_ej0.txt)
# round 5: the gate GEMM's column statistics as sums only (production) against
# sums + sums of squares (build_var/libold.so: the sources before the change):
# gate / C5 tests, tools/gate_bench.py, then C5 bench legs new / old / new / old
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_vit_block.py tests/test_c5_gpu.py tests/test_pgemm_gpu.py tests/test_fused_gpu.py > gpurun_out/r5_sumonly_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/r5_sumonly_tests.log; [ $rc = 0 ] || exit 1
for v in new old; do
  if [ $v = new ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libold.so; fi
  ARTSBIR_TUNE_CACHE=$R/profiles/tune_r5.txt timeout -k 10 300 python -u tools/gate_bench.py > gpurun_out/r5_sumonly_gate_$v.log 2>&1 || { echo FAILED; exit 1; }
  echo "== $v"; grep run gpurun_out/r5_sumonly_gate_$v.log
done
B="python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2"
i=0
for v in new old new old; do
  i=$((i+1))
  if [ $v = new ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libold.so; fi
  timeout -k 10 600 $B > gpurun_out/r5_sumonly_$i.json 2>gpurun_out/r5_sumonly_$i.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_sumonly_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_sumonly_$i.json').read().strip().splitlines()[-1]); print('$v c2', d['ms_per_step'], 'c5', d['c5']['ms_per_step'])"
done
