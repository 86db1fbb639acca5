#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-profile --steps 3 --warmup 2"
timeout -k 10 300 $B > gpurun_out/ab3_notune.json 2>/dev/null || exit 1
timeout -k 10 300 $B --tune-cache profiles/tune_r2.txt > gpurun_out/ab3_cache.json 2>/dev/null || exit 1
for v in notune cache; do python3 -c "import json; d=json.loads(open('gpurun_out/ab3_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['allocator'])"; done
