#!/bin/bash
# (measured neutral: the VT_/AT_/Q_NT_STORE knobs were removed again; the script needs them back)
# round 4: non-temporal stores in the ViT elementwise kernels, the attention
# outputs and the fp8 quantiser codes (diagnostic build
# art-sbir_amd/build_var/libvnt.so: -DVT_NT_STORE=1 -DAT_NT_STORE=1 -DQ_NT_STORE=1)
# against the production build (fp8 GEMM stores non-temporal in both): C5 steps, alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in base nt base nt; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libvnt.so; fi
  echo "== $v $(ARTSBIR_TUNE_CACHE=profiles/tune_r4.txt timeout -k 10 300 python3 tools/c5_step.py 512 fp8 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
done
