#!/bin/bash
# round 4: weight-gradient scheduling knobs re-measured with the pw256 / pp256 table (C2 leg only, 2 rounds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-loss-check --no-profile --steps 10 --warmup 3 > gpurun_out/r4_sched.json 2> gpurun_out/r4_sched.err || { echo "FAIL $1"; tail -5 gpurun_out/r4_sched.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r4_sched.json').read().strip().splitlines()[-1]);print('$1', d['ms_per_step'], d['value'])"
}
for r in 1 2; do
  for k in BASE=1 ARTSBIR_WGRAD_MAIN=3x3 ARTSBIR_WGRAD_MAIN=1x1 ARTSBIR_WGRAD_DEFER=3x3 ARTSBIR_WGRAD_DEFER=1x1 ARTSBIR_SIDE_CUS=64 ARTSBIR_SIDE_CUS=128; do
    run $k || exit 1
  done
done
