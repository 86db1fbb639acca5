#!/bin/bash
# round 6: the gated GEMM's first-round stagger (ARTSBIR_PP_STAGGER = n x s_sleep(127)
# for alternate CUs' first tiles) — gate_bench at n = 0 / 3 / 6 / 10, then C5 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for n in 0 3 6 10; do
    echo -n "stagger $n: "; ARTSBIR_PP_STAGGER=$n timeout -k 10 120 python -u tools/gate_bench.py 2>&1 | grep '"gate+sums"' || exit 1
  done
done
