#!/bin/bash
# full bench (training leg) under several environment settings: args "name:VAR=val,VAR2=val"
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-retrieval --steps 8 > gpurun_out/env_$name.json 2> gpurun_out/env_$name.err || { echo BENCH_FAILED; tail -20 gpurun_out/env_$name.err; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/env_$name.json)"
done
