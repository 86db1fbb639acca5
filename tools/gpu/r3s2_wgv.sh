#!/bin/bash
# A/B of weight-gradient tile / split choices inside the overlapped C2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for t in profiles/tune_r3s2.txt scratch_wgv/v1.txt scratch_wgv/v2.txt scratch_wgv/v3.txt scratch_wgv/v4.txt profiles/tune_r3s2.txt; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $t > gpurun_out/wgv_out.json 2> gpurun_out/wgv_out.err || { echo FAIL $t; tail -5 gpurun_out/wgv_out.err; exit 1; }
  python -c "import json,sys; l=json.load(open('gpurun_out/wgv_out.json')); print(sys.argv[1], l['value'], l['ms_per_step'], l['allocator']['step_ms'])" $t
done
