#!/bin/bash
# round 4: the fp8 quantiser with four 16-B loads in flight per lane (production)
# against one (diagnostic build art-sbir_amd/build_var/libq1.so, the previous
# fp8.hip): ViT fp8 parity tests, then C5 steps alternated with kernel averages
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_block.py tests/test_c5_gpu.py -m gpu > gpurun_out/r4_q4_tests.log 2>&1 || { tail -30 gpurun_out/r4_q4_tests.log; exit 1; }
tail -1 gpurun_out/r4_q4_tests.log
for v in q1 q4 q1 q4; do
  if [ $v = q4 ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  echo "== $v"
  ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
