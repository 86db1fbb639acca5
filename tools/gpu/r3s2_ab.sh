#!/bin/bash
# session-2: GPU tests of the changed kernels, then the C2 leg with the committed
# table (GLB epilogue batch EJB=2 in this build; EJB=1 numbers in profiles/r3s2_c2_tuned_bench.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py tests/test_encoder_gpu.py tests/test_c2_gpu.py tests/test_modules_gpu.py -q -rf --timeout 400 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/s2_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_ab.json 2> gpurun_out/s2_ab.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_ab.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/s2_ab.json').read().strip().splitlines()[-1])
print("value", d['value'], "ms", d['ms_per_step'], "steps", d['allocator']['step_ms'])
pk=d['roofline']['per_kernel']
for k,v in sorted(pk.items(), key=lambda kv:-kv[1]['share_s'])[:12]:
    print(f"{v['share_s']*1e3/d['steps']:8.2f} ms/step {v['launches']/d['steps']:6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {v['gbs']:7.1f}GB/s {k}")
PY
