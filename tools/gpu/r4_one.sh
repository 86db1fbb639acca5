#!/bin/bash
# round 4: pp256 schedule A/B: two 16-MFMA phases per K-tile (production) vs one 32-MFMA phase
# (diagnostic build art-sbir_amd/build_var/libone.so), NT and conv shapes, parity of the variant first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ARTSBIR_LIB=$R/art-sbir_amd/build_var/libone.so timeout -k 10 300 python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "22 or pp256" -p no:cacheprovider > gpurun_out/r4_one_t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r4_one_t.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
for v in prod one; do
  lib=""; [ $v = one ] && lib="ARTSBIR_LIB=$R/art-sbir_amd/build_var/libone.so"
  echo "== $v"
  env $lib timeout -k 10 300 python -u tools/pp_bench.py --cands 22 --rounds 1 > gpurun_out/r4_one_$v.log 2>&1 || { echo FAIL; tail -3 gpurun_out/r4_one_$v.log; exit 1; }
  grep -E "^nt|^conv" gpurun_out/r4_one_$v.log | awk '{printf "%s %s %s %s\n", $1, $2, $5, $8}'
done
done
