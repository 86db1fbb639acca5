#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for d in 0 1 4 8 9 13; do
  echo "#### ARTSBIR_PG_DBG=$d"
  ARTSBIR_PG_DBG=$d CFGS=0,1 timeout -k 10 200 python -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
