#!/bin/bash
# round-2 check on the GPU box: new C2 parity + retrieval tests, the rest of the
# GPU suite, then one bench line (tune cache saved for the profiled re-runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }   # pytest: 0 pass, 1 test failures; anything else = stop
timeout -k 10 600 python -u -m pytest tests/test_c2_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/c2.log 2>&1; rc=$?
echo "c2 rc=$rc"; grep -E "PASS|FAIL|ERROR|C2 bf16|passed|failed" gpurun_out/c2.log | tail -20
ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py -q -rf --timeout 300 --timeout-method thread > gpurun_out/retr.log 2>&1; rc=$?
echo "retr rc=$rc"; tail -15 gpurun_out/retr.log
ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread --deselect tests/test_c2_gpu.py --ignore tests/test_retrieval_gpu.py --ignore tests/test_c2_gpu.py > gpurun_out/gpu_rest.log 2>&1; rc=$?
echo "rest rc=$rc"; tail -8 gpurun_out/gpu_rest.log
ok $rc || exit $rc
timeout -k 10 900 python -u bench.py --tune-cache gpurun_out/tune_c2.txt > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cut -c1-1500 gpurun_out/bench.json
