#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for U in 1 3 9; do
  echo "== lib u$U"
  ARTSBIR_LIB=$PWD/scratch/libs/lib_u$U.so SHAPES=stem3_dg,stem2_dg,l1_act3x3,stem2_fwd,stem3_fwd,l1_fwd CFGS=21 timeout -k 10 200 python -u scratch/epi_bench.py > gpurun_out/hconv_u$U.txt 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/hconv_u$U.txt; exit 1; }
  grep -v "amdgpu.ids\|copy" gpurun_out/hconv_u$U.txt
done
