#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for P in 0 -1; do
ARTSBIR_STEP_PRIO=$P timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-retrieval > gpurun_out/bench_prio$P.json 2> gpurun_out/bench_prio$P.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_prio$P.err; exit 1; }
echo "prio $P"; cut -c1-330 gpurun_out/bench_prio$P.json | grep -o '"ms_per_step": [0-9.]*'
done
