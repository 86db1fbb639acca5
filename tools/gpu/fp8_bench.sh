#!/bin/bash
# fp8 projection GEMM variants at the C5 bench's token count; args: configs (default 0 3)
set -e
mkdir -p gpurun_out
cfgs=${@:-0 3}
for cfg in $cfgs; do
  ARTSBIR_FP8_CFG=$cfg timeout -k 10 120 python -u tools/fp8_bench.py >> gpurun_out/fp8_bench.txt 2>&1
  ARTSBIR_FP8_CFG=$cfg ARTSBIR_FP8_NOSTORE=1 timeout -k 10 120 python -u tools/fp8_bench.py >> gpurun_out/fp8_bench.txt 2>&1
done
grep -v amdgpu.ids gpurun_out/fp8_bench.txt
