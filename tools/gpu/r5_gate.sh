#!/bin/bash
# round 5: cost of the QuickGELU gate and the column-sum slots in the C5 c_proj
# data gradient (tools/gate_bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ARTSBIR_TUNE_CACHE=$R/profiles/tune_r5.txt timeout -k 10 300 python -u tools/gate_bench.py > gpurun_out/r5_gate.log 2>&1 || { echo FAILED; tail -5 gpurun_out/r5_gate.log; exit 1; }
grep run gpurun_out/r5_gate.log
