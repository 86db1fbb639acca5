#!/bin/bash
# round 6: re-tune every C2 shape with the new candidates (26: the streaming RES
# data gradient), save the table, then the C2 leg on the new and the old table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-loss-check"
timeout -k 10 600 python -u bench.py $C2 --steps 3 --warmup 2 --tune-cache none --tune-save gpurun_out/tune_r6.txt > gpurun_out/r6_retune.log 2>&1 || { echo RETUNE_FAILED; tail -5 gpurun_out/r6_retune.log; exit 1; }
grep -c . gpurun_out/tune_r6.txt; awk '$17==26' gpurun_out/tune_r6.txt
for t in gpurun_out/tune_r6.txt profiles/tune_r5.txt gpurun_out/tune_r6.txt; do
  timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 --tune-cache $t > gpurun_out/r6_tab.log 2>&1 || { echo RUN_FAILED; tail -5 gpurun_out/r6_tab.log; exit 1; }
  tail -1 gpurun_out/r6_tab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['value'], d['roofline']['streams_kernel_ms'])"
done
