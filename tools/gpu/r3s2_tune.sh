#!/bin/bash
# session-2: re-tune the conv choices (new candidates 16 / 17) with the committed
# weight-gradient choices kept, save the merged table, then time the C2 leg with it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fused_gpu.py tests/test_pgemm_gpu.py -q -rf --timeout 300 --timeout-method thread -k "17 or 16" > gpurun_out/s2_cand.log 2>&1; rc=$?
echo "cand tests rc=$rc"; tail -3 gpurun_out/s2_cand.log; [ $rc = 0 ] || exit 1
grep -v '^c ' profiles/tune_r3.txt > gpurun_out/s2_tune_wonly.txt
summ() {
python3 - "$1" <<'PY'
import json, sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", d['value'], "ms", d['ms_per_step'], "steps", d['allocator']['step_ms'])
pk=d['roofline']['per_kernel']
for k,v in sorted(pk.items(), key=lambda kv:-kv[1]['share_s'])[:22]:
    print(f"{v['share_s']*1e3/d['steps']:8.2f} ms/step {v['launches']/d['steps']:6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {v['gbs']:7.1f}GB/s {k}")
PY
}
timeout -k 10 600 python -u bench.py --no-cpu-baseline --tune-cache gpurun_out/s2_tune_wonly.txt --tune-save gpurun_out/s2_tune_all.txt > gpurun_out/s2_tune_run.json 2> gpurun_out/s2_tune_run.err || { echo TUNE_RUN_FAILED; tail -20 gpurun_out/s2_tune_run.err; exit 1; }
summ gpurun_out/s2_tune_run.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --tune-cache gpurun_out/s2_tune_all.txt > gpurun_out/s2_tuned.json 2> gpurun_out/s2_tuned.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_tuned.err; exit 1; }
summ gpurun_out/s2_tuned.json
