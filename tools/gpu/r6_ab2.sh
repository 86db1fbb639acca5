#!/bin/bash
# round 6: A/B of one engine change on the C2 leg (same box, interleaved runs)
#   ARGS: the env assignment of the B runs, e.g. ARTSBIR_X=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-loss-check"
for i in 1 2; do
  for v in A B; do
    if [ $v = B ]; then E="$1"; else E=""; fi
    env $E timeout -k 10 300 python -u bench.py $C2 --steps 10 --warmup 3 > gpurun_out/r6_ab_$v.log 2>&1 || { echo RUN_FAILED; tail -5 gpurun_out/r6_ab_$v.log; exit 1; }
    tail -1 gpurun_out/r6_ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['value'], d['roofline']['streams_kernel_ms'])"
  done
done
