#!/bin/bash
# round 5: the committed tuning table vs the same with the non-temporal forward
# candidates on the 28^2 / 14^2 / 7^2 1x1 statistics forwards (profiles/tune_r5_nt.txt), alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-profile --steps 10 --warmup 3"
for i in 1 2; do
  for t in tune_r5 tune_r5_nt; do
    timeout -k 10 300 $B --tune-cache profiles/$t.txt > gpurun_out/r5_ntab_${t}_$i.json 2>/dev/null || { echo FAIL $t; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5_ntab_${t}_$i.json').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'])"
  done
done
