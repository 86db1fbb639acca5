#!/bin/bash
# session-2 iteration: quick parity tests (+ the new fused-dgrad candidate), the C2
# bench leg with the committed tune table and re-tuned (new candidates), tables saved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu/tests_quick.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py -q -rf --timeout 300 --timeout-method thread -k "dgrad_fused_bn_reduce and (16 or auto)" > gpurun_out/s2_fused16.log 2>&1; rc=$?
echo "fused16 rc=$rc"; tail -3 gpurun_out/s2_fused16.log; [ $rc = 0 ] || exit 1
summ() {
python3 - "$1" <<'PY'
import json, sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", d['value'], "ms", d['ms_per_step'], "steps", d['allocator']['step_ms'])
pk=d['roofline']['per_kernel']
for k,v in sorted(pk.items(), key=lambda kv:-kv[1]['share_s'])[:24]:
    print(f"{v['share_s']*1e3/d['steps']:8.2f} ms/step {v['launches']/d['steps']:6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {v['gbs']:7.1f}GB/s {k}")
PY
}
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_iter_a.json 2> gpurun_out/s2_iter_a.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_iter_a.err; exit 1; }
summ gpurun_out/s2_iter_a.json
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache none --tune-save gpurun_out/s2_tune_c2.txt > gpurun_out/s2_iter_b.json 2> gpurun_out/s2_iter_b.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_iter_b.err; exit 1; }
summ gpurun_out/s2_iter_b.json
