#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-profile --steps 6 --warmup 2"
timeout -k 10 300 $B > gpurun_out/al_a.json 2>/dev/null || exit 1
timeout -k 10 300 $B --tune-cache profiles/tune_r2.txt > gpurun_out/al_b.json 2>/dev/null || exit 1
timeout -k 10 300 $B --tune-cache profiles/tune_r2.txt > gpurun_out/al_c.json 2>/dev/null || exit 1
for v in a b c; do python3 -c "import json; d=json.loads(open('gpurun_out/al_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['allocator'])"; done
