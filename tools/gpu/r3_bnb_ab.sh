#!/bin/bash
# C2 step with the fused BN-backward dgrads forced to one candidate (A/B of the tuner's quiet-device choice)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for cfg in none 14 3 0; do
  if [ $cfg = none ]; then unset ARTSBIR_BNB_CFG; else export ARTSBIR_BNB_CFG=$cfg; fi
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-embed --no-c5 --no-retrieval --no-preprocess \
    --no-cpu-baseline --no-loss-check --no-profile > gpurun_out/r3_bnb_$cfg.json 2> gpurun_out/r3_bnb_$cfg.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r3_bnb_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', d['ms_per_step'], d['allocator']['step_ms'])"
done
