#!/bin/bash
# A/B of two library builds on the full bench (training leg only)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for L in "$@"; do
ARTSBIR_LIB=$R/scratch/libs/$L.so ARTSBIR_STEP_PRIO=-1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-retrieval --steps 8 > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || { echo BENCH_FAILED; tail -20 gpurun_out/ab_$L.err; exit 1; }
echo "$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$L.json)"
done
