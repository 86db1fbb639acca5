#!/bin/bash
# A/B: step time with the autotune cache loaded vs tuned in-process
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-profile --steps 5 --warmup 2"
for v in "notune" "cache" "cache_noloss" "notune_full"; do
  case $v in
    notune) A="";;
    cache) A="--tune-cache profiles/tune_r2.txt";;
    cache_noloss) A="--tune-cache profiles/tune_r2.txt --no-loss-check";;
    notune_full) A="--no-loss-check";;
  esac
  timeout -k 10 300 $B $A > gpurun_out/ab_$v.json 2>/dev/null || { echo FAIL $v; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
done
