#!/bin/bash
# session-2: candidate 19 (256x128 8-wave tile, 32-k stages, 2 workgroups per CU)
# for the plain / statistics / bias-ReLU epilogues: parity tests, then the full
# bench with every non-BN-backward conv key re-tuned (same box A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_fused_gpu.py -q -rf --timeout 300 --timeout-method thread -k "19 or auto" > gpurun_out/s2_c19_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s2_c19_tests.log; [ $rc = 0 ] || exit 1
awk '!($1=="c" && $16=="0" && !($3=="1" && $4=="1"))' profiles/tune_r3s2.txt > gpurun_out/s2_tune_noplain.txt
for t in profiles/tune_r3s2.txt gpurun_out/s2_tune_noplain.txt gpurun_out/s2_tune_c19.txt; do
  save=""; [ $t = gpurun_out/s2_tune_noplain.txt ] && save="--tune-save gpurun_out/s2_tune_c19.txt"
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-c5 --no-retrieval --no-preprocess --tune-cache $t $save > gpurun_out/s2_c19.json 2> gpurun_out/s2_c19.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_c19.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s2_c19.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel']
print('$t', d['value'], d['ms_per_step'], d['allocator']['step_ms'], 'embed', d['embed']['value'], {k:(v['launches']/d['steps'], v['avg_us']) for k,v in pk.items() if 'glb>' in k or k.startswith('pstream_kernel<128>')})"
done
awk '$1=="c" && $17=="19"' gpurun_out/s2_tune_c19.txt | head -30
