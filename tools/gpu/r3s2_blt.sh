#!/bin/bash
# session-2: hipBLASLt candidate (-3) for the plain dense GEMMs: its parity test,
# then C2 + C5 legs with the committed table and with the dense-GEMM entries
# re-tuned (-3 competing), same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pgemm_gpu.py tests/test_gemm_gpu.py -q -rf --timeout 300 --timeout-method thread -k "hipblaslt or gemm_nt" > gpurun_out/s2_blt_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/s2_blt_tests.log; [ $rc = 0 ] || exit 1
awk '!($1=="c" && $3=="1" && $4=="1")' profiles/tune_r3s2.txt > gpurun_out/s2_tune_nodense.txt
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
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess > gpurun_out/s2_blt_a.json 2> gpurun_out/s2_blt_a.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_blt_a.err; exit 1; }
summ gpurun_out/s2_blt_a.json
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-embed --no-retrieval --no-preprocess --tune-cache gpurun_out/s2_tune_nodense.txt --tune-save gpurun_out/s2_tune_blt.txt > gpurun_out/s2_blt_b.json 2> gpurun_out/s2_blt_b.err || { echo BENCH_FAILED; tail -20 gpurun_out/s2_blt_b.err; exit 1; }
summ gpurun_out/s2_blt_b.json
