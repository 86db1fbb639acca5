#!/bin/bash
# session-2: hipBLASLt candidate with an f32 bias epilogue (the attention-pool
# k|v projection): parity tests, then the C2 leg with that key re-tuned
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_c2_gpu.py -q -rf --timeout 300 --timeout-method thread -k "hipblaslt or bias or c2_bf16" > gpurun_out/s2_bltb_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s2_bltb_tests.log; [ $rc = 0 ] || exit 1
awk '!($1=="c" && $3=="1" && $4=="1" && $14=="2")' profiles/tune_r3s2.txt > gpurun_out/s2_tune_nobias.txt
for t in profiles/tune_r3s2.txt gpurun_out/s2_tune_nobias.txt; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $t --tune-save gpurun_out/s2_tune_bltb.txt > gpurun_out/s2_bltb.json 2> gpurun_out/s2_bltb.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_bltb.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s2_bltb.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel']
print('$t', d['value'], d['ms_per_step'], d['allocator']['step_ms'], {k:(v['launches']/d['steps'], v['avg_us']) for k,v in pk.items() if 'blas' in k or k=='pgemm_kernel<256,256>'})"
done
grep '^c 57600' gpurun_out/s2_tune_bltb.txt
