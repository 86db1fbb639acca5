#!/bin/bash
# session-2: attention key-side backward in two passes (one accumulator pair
# live, 128 VGPRs, two workgroups per CU): parity tests, then C2 + C5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_vit_block.py tests/test_c5_gpu.py -q -rf --timeout 400 --timeout-method thread > gpurun_out/s2_attn_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s2_attn_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_attn.json 2> gpurun_out/s2_attn.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_attn.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/s2_attn.json').read().strip().splitlines()[-1])
c5=d['c5']; print("C2", d['value'], d['ms_per_step'], "| C5", c5['value'], c5['ms_per_step'])
for k,v in sorted(c5['roofline']['per_kernel'].items(), key=lambda kv:-kv[1]['share_s'])[:7]:
    print(f"   {v['share_s']*1e3/c5['steps']:8.2f} ms/step {v['launches']/c5['steps']:6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {k}")
PY
