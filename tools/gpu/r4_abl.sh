#!/bin/bash
# round 4: pp256 timing ablations of the lean loop (diagnostic builds art-sbir_amd/build_var/libabl{1,2,3}.so:
# 1 no stage loads in the loop, 2 no fragment reads, 3 neither), NT shapes, wrong results by design
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in 0 1 2 3; do
  lib=""; [ $v != 0 ] && lib="ARTSBIR_LIB=$R/art-sbir_amd/build_var/libabl$v.so"
  echo "== abl $v"
  env $lib timeout -k 10 200 python -u tools/pp_bench.py --cands 22 --rounds 1 --only nt > gpurun_out/r4_abl_$v.log 2>&1 || { echo FAIL; tail -3 gpurun_out/r4_abl_$v.log; exit 1; }
  grep "^nt" gpurun_out/r4_abl_$v.log | awk '{print $2, $6, $7, $8}'
done
