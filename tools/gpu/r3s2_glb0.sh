#!/bin/bash
# session-2: GLB candidate 16 for plain residual / gate epilogues: parity tests,
# then C2 + C5 with the dense / gate / residual-dgrad entries re-tuned
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_pgemm_gpu.py tests/test_vit_block.py tests/test_fused_gpu.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/s2_glb0_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s2_glb0_tests.log; [ $rc = 0 ] || exit 1
awk '!($1=="c" && (($3=="1" && $4=="1") || ($13!="0" && $16=="0")))' profiles/tune_r3s2.txt > gpurun_out/s2_tune_base.txt
summ() {
python3 - "$1" <<'PY'
import json, sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c5=d.get('c5',{})
print(sys.argv[1], "C2", d['value'], d['ms_per_step'], "| C5", c5.get('value'), c5.get('ms_per_step'))
pk=c5.get('roofline',{}).get('per_kernel',{})
for k,v in sorted(pk.items(), key=lambda kv:-kv[1]['share_s'])[:8]:
    print(f"   {v['share_s']*1e3/c5.get('steps',2):8.2f} ms/step {v['launches']/c5.get('steps',2):6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {k}")
PY
}
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --tune-cache gpurun_out/s2_tune_base.txt --tune-save gpurun_out/s2_tune_glb0.txt > gpurun_out/s2_glb0.json 2> gpurun_out/s2_glb0.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_glb0.err; exit 1; }
summ gpurun_out/s2_glb0.json
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --tune-cache gpurun_out/s2_tune_glb0.txt > gpurun_out/s2_glb0b.json 2> gpurun_out/s2_glb0b.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_glb0b.err; exit 1; }
summ gpurun_out/s2_glb0b.json
