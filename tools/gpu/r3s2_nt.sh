#!/bin/bash
# session-2 A/B: non-temporal last-read loads in bn_bwd_apply (default build) vs
# plain loads (libartsbir_hip_nt0.so), C2 leg alternated on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_c2_gpu.py tests/test_fused_gpu.py -q -rf --timeout 300 --timeout-method thread -k "c2 or forward_branches or triplet" > gpurun_out/s2_nt_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/s2_nt_tests.log; [ $rc = 0 ] || exit 1
for v in nt nt0 nt nt0; do
  lib=$R/art-sbir_amd/libartsbir_hip.so; [ $v = nt0 ] && lib=$R/art-sbir_amd/libartsbir_hip_nt0.so
  ARTSBIR_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_nt_$v.json 2> gpurun_out/s2_nt_$v.err || { echo BENCH_FAILED $v; tail -20 gpurun_out/s2_nt_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s2_nt_$v.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel']; a=pk.get('bn_bwd_apply_kernel<2>',{})
print('$v', d['value'], d['ms_per_step'], d['allocator']['step_ms'], 'apply2', a.get('avg_us'), a.get('gbs'))"
done
