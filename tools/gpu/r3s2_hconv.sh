#!/bin/bash
# session-2: halo-conv kernel with three halo buffers / BN operand one tile ahead:
# its parity tests, then the C2 leg (committed table)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py tests/test_encoder_gpu.py -q -rf --timeout 400 --timeout-method thread > gpurun_out/s2_hc_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s2_hc_tests.log; [ $rc = 0 ] || exit 1
bash tools/gpu/tests_quick.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_hc.json 2> gpurun_out/s2_hc.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_hc.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/s2_hc.json').read().strip().splitlines()[-1])
print("value", d['value'], "ms", d['ms_per_step'], "steps", d['allocator']['step_ms'])
pk=d['roofline']['per_kernel']
for k,v in sorted(pk.items(), key=lambda kv:-kv[1]['share_s'])[:40]:
    if 'hconv' in k or v['share_s']*1e3/d['steps'] > 5:
        print(f"{v['share_s']*1e3/d['steps']:8.2f} ms/step {v['launches']/d['steps']:6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {v['gbs']:7.1f}GB/s {k}")
PY
