#!/bin/bash
# session-2: register-prefetched epilogue candidates (11-13) for the gated GEMM
# (C5 c_proj input gradient): parity tests, then C5 with that key re-tuned
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vit_block.py -q -rf --timeout 300 --timeout-method thread -k "gate" > gpurun_out/s2_gate_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s2_gate_tests.log; [ $rc = 0 ] || exit 1
awk '!($1=="c" && $13=="3")' profiles/tune_r3s2.txt > gpurun_out/s2_tune_nogate.txt
for t in profiles/tune_r3s2.txt gpurun_out/s2_tune_nogate.txt; do
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --tune-cache $t --tune-save gpurun_out/s2_tune_gate.txt > gpurun_out/s2_gate.json 2> gpurun_out/s2_gate.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_gate.err; exit 1; }
  python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/s2_gate.json').read().strip().splitlines()[-1])
c5=d['c5']; print("C2", d['value'], d['ms_per_step'], "| C5", c5['value'], c5['ms_per_step'])
for k,v in sorted(c5['roofline']['per_kernel'].items(), key=lambda kv:-kv[1]['share_s'])[:6]:
    print(f"   {v['share_s']*1e3/c5['steps']:8.2f} ms/step {v['launches']/c5['steps']:6.1f} {v['avg_us']:8.1f}us {v['tflops']:7.1f}TF {k}")
PY
done
grep '^c .* 3 1 1 0 ' gpurun_out/s2_tune_gate.txt
