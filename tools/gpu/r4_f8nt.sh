#!/bin/bash
# (F8_NT_STORE is now the default; the old base is -DF8_NT_STORE=0)
# round 4: non-temporal epilogue stores in the fp8 projection GEMM (diagnostic
# build art-sbir_amd/build_var/libf8nt.so, hipcc -DF8_NT_STORE=1 on fp8.hip):
# tools/fp8_bench.py and C5 steps, alternated with the production build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in base nt base nt; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libf8nt.so; fi
  echo "== $v"
  timeout -k 10 120 python3 tools/fp8_bench.py 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,json;[print(' ',l.strip()) for l in sys.stdin if 'total' in l or 'gemm' in l]" || exit 1
  ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
