#!/bin/bash
# round 5: re-tune every leg's kernel choices on the round-5 kernels (fold,
# layer-1 one-pass, GLB epilogue order) into profiles/tune_r5b.txt, then the
# default bench line with that table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_pgemm_gpu.py > gpurun_out/r5_pgemm_tests.log 2>&1; rc=$?
echo "pgemm tests rc=$rc"; tail -2 gpurun_out/r5_pgemm_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 1000 python -u bench.py --no-cpu-baseline --tune-cache none --tune-save gpurun_out/tune_r5b.txt --steps 3 --warmup 2 > gpurun_out/r5_retune.json 2> gpurun_out/r5_retune.err || { echo TUNE_FAILED; tail -20 gpurun_out/r5_retune.err; exit 1; }
wc -l gpurun_out/tune_r5b.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline --tune-cache gpurun_out/tune_r5b.txt > gpurun_out/r5_bench_b.json 2> gpurun_out/r5_bench_b.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5_bench_b.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r5_bench_b.json",):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], "c5", d["c5"]["ms_per_step"], "embed", d["embed"]["value"], "retr", d["retrieval"]["ms"])
PY
