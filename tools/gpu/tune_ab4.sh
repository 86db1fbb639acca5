#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-profile --steps 4 --warmup 2 --tune-cache profiles/tune_r2.txt"
timeout -k 10 300 $B > gpurun_out/ab4_a.json 2>/dev/null || exit 1
timeout -k 10 300 $B --sync-warmup > gpurun_out/ab4_b.json 2>/dev/null || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 300 $B > gpurun_out/ab4_c.json 2>/dev/null || exit 1
for v in a b c; do python3 -c "import json; d=json.loads(open('gpurun_out/ab4_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['allocator'])"; done
