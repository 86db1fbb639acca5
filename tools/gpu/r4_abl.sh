#!/bin/bash
# round 4: pp256 timing ablations (ARTSBIR_PG_DBG bits, wrong results by design) on the NT shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for d in 0 8 16 24 32 40 56; do
  echo "== dbg $d"
  ARTSBIR_PG_DBG=$d timeout -k 10 200 python -u tools/pp_bench.py --cands 0,22 --rounds 1 --only nt > gpurun_out/r4_abl_$d.log 2>&1 || { echo FAIL; tail gpurun_out/r4_abl_$d.log; exit 1; }
  grep "x2304 \|x768x3072\|57600" gpurun_out/r4_abl_$d.log
done
