#!/bin/bash
# session-2 A/B: weight gradients of one class (1x1 / 3x3) in order on the main
# stream instead of the side stream (ARTSBIR_WGRAD_MAIN), C2 leg, same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for mode in none 1x1 3x3 none; do
  ARTSBIR_WGRAD_MAIN=$([ $mode = none ] && echo "" || echo $mode) timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-profile > gpurun_out/s2_wgm_$mode.json 2> gpurun_out/s2_wgm_$mode.err || { echo BENCH_FAILED $mode; tail -20 gpurun_out/s2_wgm_$mode.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s2_wgm_$mode.json').read().strip().splitlines()[-1])
print('$mode', d['value'], d['ms_per_step'], d['allocator']['step_ms'])"
done
