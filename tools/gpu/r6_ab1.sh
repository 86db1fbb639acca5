#!/bin/bash
# round 6: C2 leg with bn1 folded through conv1 vs the apply pass (same box),
# the first run saving the tune table with the new fold_y shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-loss-check"
timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 --tune-save gpurun_out/tune_r6.txt > gpurun_out/r6_ab1_on.log 2>&1 || { echo ON_FAILED; tail -5 gpurun_out/r6_ab1_on.log; exit 1; }
tail -1 gpurun_out/r6_ab1_on.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fold1 on ', d['ms_per_step'], d['value'])"
ARTSBIR_FOLD_BN1=0 timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 --tune-cache gpurun_out/tune_r6.txt > gpurun_out/r6_ab1_off.log 2>&1 || { echo OFF_FAILED; tail -5 gpurun_out/r6_ab1_off.log; exit 1; }
tail -1 gpurun_out/r6_ab1_off.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fold1 off', d['ms_per_step'], d['value'])"
timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 --tune-cache gpurun_out/tune_r6.txt > gpurun_out/r6_ab1_on2.log 2>&1 || { echo ON2_FAILED; tail -5 gpurun_out/r6_ab1_on2.log; exit 1; }
tail -1 gpurun_out/r6_ab1_on2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fold1 on ', d['ms_per_step'], d['value'])"
