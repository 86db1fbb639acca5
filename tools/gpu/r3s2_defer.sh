#!/bin/bash
# A/B inside the C2 step: weight gradients issued beside their layer's data
# gradient (default) or held until it has run (ARTSBIR_WGRAD_DEFER), then the
# C2 parity tests with every weight gradient deferred
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for d in none 3x3 1x1 all none 3x3 all; do
  v=$d; [ $d = none ] && v=
  ARTSBIR_WGRAD_DEFER=$v timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/defer_out.json 2> gpurun_out/defer_out.err || { echo FAIL $d; tail -5 gpurun_out/defer_out.err; exit 1; }
  python -c "import json,sys; l=json.load(open('gpurun_out/defer_out.json')); print(sys.argv[1], l['value'], l['ms_per_step'], l['allocator']['step_ms'])" $d
done
ARTSBIR_WGRAD_DEFER=all timeout -k 10 600 python -u -m pytest tests/test_c2_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/defer_tests.log 2>&1; rc=$?
tail -2 gpurun_out/defer_tests.log; exit $rc
