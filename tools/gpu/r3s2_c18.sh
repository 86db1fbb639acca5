#!/bin/bash
# session-2: candidate 18 (256x128 GLB fused RES dgrad, 2 workgroups per CU):
# parity tests, then the C2 leg with the kind-3 dgrad keys re-tuned (same box A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py -q -rf --timeout 300 --timeout-method thread -k "18 or auto" > gpurun_out/s2_c18_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s2_c18_tests.log; [ $rc = 0 ] || exit 1
awk '!($1=="c" && ($16=="13" || $16=="14"))' profiles/tune_r3s2.txt > gpurun_out/s2_tune_nok3.txt
for t in profiles/tune_r3s2.txt gpurun_out/s2_tune_nok3.txt gpurun_out/s2_tune_c18.txt; do
  save=""; [ $t = gpurun_out/s2_tune_nok3.txt ] && save="--tune-save gpurun_out/s2_tune_c18.txt"
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $t $save > gpurun_out/s2_c18.json 2> gpurun_out/s2_c18.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_c18.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s2_c18.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel']
print('$t', d['value'], d['ms_per_step'], d['allocator']['step_ms'], {k:(v['launches']/d['steps'], v['avg_us']) for k,v in pk.items() if 'bnb' in k and 'pgemm' in k})"
done
awk '$1=="c" && ($16=="13" || $16=="14")' gpurun_out/s2_tune_c18.txt
