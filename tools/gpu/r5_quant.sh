#!/bin/bash
# round 5: fp8 quantiser variants (build_var/libq{w16,nt,w16nt}.so: 16 values per
# lane / non-temporal stores / both) against production: the exhaustive code test
# on each, then tools/quant_bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
for v in base w16 nt w16nt; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libq$v.so; fi
  timeout -k 10 300 $T tests/test_vit_block.py -k "fp8" > gpurun_out/r5_quant_tests_$v.log 2>&1 || { echo "TESTS_FAILED $v"; tail -5 gpurun_out/r5_quant_tests_$v.log; exit 1; }
  timeout -k 10 300 python -u tools/quant_bench.py > gpurun_out/r5_quant_$v.log 2>&1 || { echo "BENCH_FAILED $v"; tail -5 gpurun_out/r5_quant_$v.log; exit 1; }
  echo "== $v $(tail -1 gpurun_out/r5_quant_tests_$v.log)"; cat gpurun_out/r5_quant_$v.log | grep shape
done
