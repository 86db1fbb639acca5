#!/bin/bash
# C2 step with the fused BN-backward dgrads forced to one tile configuration
# (args: configs; "t" = autotuned) — does a smaller-LDS dgrad co-reside with
# the side-stream weight gradients better than the standalone-fastest one?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in ${@:-t 3 13}; do
  if [ "$c" = t ]; then unset ARTSBIR_BNB_CFG; else export ARTSBIR_BNB_CFG=$c; fi
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-c5 --no-embed --no-retrieval --no-cpu-baseline \
    --no-loss-check --no-profile > gpurun_out/bnb_ab_$c.json 2> gpurun_out/bnb_ab_$c.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bnb_ab_$c.json').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['value'])"
done
