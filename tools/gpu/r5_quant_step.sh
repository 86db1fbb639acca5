#!/bin/bash
# round 5: the quantiser with non-temporal stores (build_var/libqnt.so) in the C5 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --no-profile --steps 3 --warmup 2"
i=0
for v in base nt base nt; do
  i=$((i+1))
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libqnt.so; fi
  timeout -k 10 600 $B > gpurun_out/r5_qstep_$i.json 2>gpurun_out/r5_qstep_$i.err || { echo BENCH_FAILED; tail -5 gpurun_out/r5_qstep_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5_qstep_$i.json').read().strip().splitlines()[-1]); print('$v c2', d['ms_per_step'], 'c5', d['c5']['ms_per_step'])"
done
