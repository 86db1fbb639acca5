#!/bin/bash
# round 5: normalize-on-load cost probe on the persistent streaming 1x1 conv
# (pstream_kernel, candidates 10 / 15) — the forward of the conv3 consumers of
# act2 (56^2 64->256 ... 7^2 512->2048, three BN segments) with the production
# build and the PG_NOL=1 diagnostic build (relu(s*x+b) on every pixel fragment,
# coefficients from LDS per 32-k step; art-sbir_amd/build_var/libnol.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in base nol; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libnol.so; fi
  echo "== $v"
  ONLY=0,1,2,3 CFGS=10,15 timeout -k 10 300 python3 -u tools/fwd_bench.py 2>&1 | grep -v "amdgpu.ids" || exit 1
done
