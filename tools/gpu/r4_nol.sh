#!/bin/bash
# round 4: cost of a consumer-side BatchNorm + ReLU on the pixel operand of the
# ping-pong tile (diagnostic build art-sbir_amd/build_var/libnol.so: pp256.hip
# with -DPP_NOL=1), candidate 22 forced on the C2 conv shapes, alternated with
# the production build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in base nol; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libnol.so; fi
  echo "== $v"
  timeout -k 10 300 python3 -u tools/pp_bench.py --cands 22 --only conv --rounds 2 2>&1 | grep -v "amdgpu.ids\|round" || exit 1
done
