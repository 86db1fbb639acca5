#!/bin/bash
# C2 step with the halo wgrad's persistent groups scaled by ARTSBIR_HW_GROUPS = 1 / 2 / 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for m in 1 2 4 1; do
  ARTSBIR_HW_GROUPS=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 10 --warmup 3 > gpurun_out/hg$m.json 2> gpurun_out/hg$m.err || { echo FAIL $m; tail -5 gpurun_out/hg$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/hg$m.json'));print('groups x$m', d['ms_per_step'], d['value'])"
done
