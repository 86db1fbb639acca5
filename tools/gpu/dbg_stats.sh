#!/bin/bash
# timing experiment: statistics reduction cost (ARTSBIR_PG_DBG bits 1 / 2) in the forward and fused dgrad kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for d in 0 1 3; do
  echo "#### ARTSBIR_PG_DBG=$d" >> gpurun_out/dbg_stats.txt
  ARTSBIR_PG_DBG=$d CFGS=0,3 timeout -k 10 200 python -u tools/fwd_bench.py 2>&1 | grep -v amdgpu.ids | grep -E "==|stats1" >> gpurun_out/dbg_stats.txt || exit 1
  ARTSBIR_PG_DBG=$d CFGS=0,3 timeout -k 10 200 python -u tools/dgrad_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/dbg_stats.txt || exit 1
done
