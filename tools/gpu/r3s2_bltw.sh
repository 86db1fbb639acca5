#!/bin/bash
# session-2: hipBLASLt as weight-gradient candidate -3 for the dense 1x1 weight
# gradients: parity tests, then the C2 bench with those keys re-tuned (same box A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py -q -rf --timeout 300 --timeout-method thread -k "wgrad_accumulates or gemm_tn_strided" > gpurun_out/s2_bltw_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s2_bltw_tests.log; [ $rc = 0 ] || exit 1
# drop the C2 dense weight-gradient keys (field 11 = dense) so they are re-tuned with -3 in the list
awk '!($1=="w" && $11=="1" && $2!="302592" && $2!="301056" && $2!="1536")' profiles/tune_r3s2.txt > gpurun_out/s2_tune_nodw.txt
for t in profiles/tune_r3s2.txt gpurun_out/s2_tune_nodw.txt gpurun_out/s2_tune_bltw.txt profiles/tune_r3s2.txt; do
  save=""; [ $t = gpurun_out/s2_tune_nodw.txt ] && save="--tune-save gpurun_out/s2_tune_bltw.txt"
  timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache $t $save > gpurun_out/s2_bltw.json 2> gpurun_out/s2_bltw.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_bltw.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s2_bltw.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel']
print('$t', d['value'], d['ms_per_step'], d['allocator']['step_ms'], {k:(v['launches']/d['steps'], v['avg_us']) for k,v in pk.items() if 'blaslt' in k})"
done
awk '$1=="w" && $15=="-3"' gpurun_out/s2_tune_bltw.txt
