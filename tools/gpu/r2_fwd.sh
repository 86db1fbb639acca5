#!/bin/bash
# forward conv microbenchmark (statistics epilogue vs none, per candidate)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CFGS=0,1,2,3,10 timeout -k 10 300 python -u tools/fwd_bench.py > gpurun_out/fwd.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fwd.txt; exit $rc
