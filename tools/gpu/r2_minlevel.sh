#!/bin/bash
# C2 step with the weight-gradient split levels restricted (ARTSBIR_WGRAD_MINLEVEL = 0 / 1 / 2 / 3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for L in 0 1 2 3; do
  ARTSBIR_WGRAD_MINLEVEL=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-profile --steps 10 --warmup 3 > gpurun_out/ml$L.json 2> gpurun_out/ml$L.err || { echo FAIL $L; tail -5 gpurun_out/ml$L.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ml$L.json'));print('minlevel $L', d['ms_per_step'], d['value'], d.get('allocator',{}).get('step_ms'))"
done
