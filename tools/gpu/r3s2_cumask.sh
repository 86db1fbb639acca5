#!/bin/bash
# weight-gradient side stream CU budget sweep on the C2 step (one process)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/cu_mask_sweep.py 0 c32 c64 c96 c128 x64 0 > gpurun_out/s2_cumask.log 2>&1
rc=$?; cat gpurun_out/s2_cumask.log | grep -v Warning; exit $rc
