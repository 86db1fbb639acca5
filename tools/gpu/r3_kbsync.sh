#!/bin/bash
# the shared-bound exchange period: KB_SYNC_TILES 8 / 32 builds against the default 16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in ${KBV:-8 32}; do
  ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib_kb$v.so ARTSBIR_KNN_STAT=1 timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r3_kb$v.log 2>&1 || { echo RETR_FAILED $v; tail -5 gpurun_out/r3_kb$v.log; exit 1; }
  echo kb$v; grep noise gpurun_out/r3_kb$v.log
done
