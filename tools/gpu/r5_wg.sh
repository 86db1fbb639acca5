#!/bin/bash
# round 5: the layer-1 fold data gradients that also accumulate their weight-
# gradient operands (artsbir_conv1x1_dgrad_fold_wg): kernel tests first, then the
# C2 / C1 / batched-branch parity tests, then the C2 step with it on and off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_fold_gpu.py -k "fold_wg" > gpurun_out/r5_wg_tests.log 2>&1; rc=$?
echo "wg tests rc=$rc"; tail -25 gpurun_out/r5_wg_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 900 $T tests/test_c2_gpu.py tests/test_c1_gpu.py tests/test_fused_gpu.py::test_forward_branches_matches_separate_calls tests/test_modules_gpu.py tests/test_encoder_gpu.py > gpurun_out/r5_wg_c2_tests.log 2>&1; rc=$?
echo "c2 tests rc=$rc"; tail -15 gpurun_out/r5_wg_c2_tests.log; [ $rc = 0 ] || exit 1
B="python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 10 --warmup 3"
timeout -k 10 400 $B > gpurun_out/r5_wg_on.json 2> gpurun_out/r5_wg_on.err || { echo BENCH_ON_FAILED; tail -20 gpurun_out/r5_wg_on.err; exit 1; }
ARTSBIR_FOLD_WG=0 timeout -k 10 400 $B > gpurun_out/r5_wg_off.json 2> gpurun_out/r5_wg_off.err || { echo BENCH_OFF_FAILED; tail -20 gpurun_out/r5_wg_off.err; exit 1; }
python - <<'PY'
import json
for n in ("on", "off"):
    d = json.loads(open(f"gpurun_out/r5_wg_{n}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(n, d["value"], d["ms_per_step"], d.get("loss_step0_rel_diff"), r.get("streams_kernel_ms"))
    for k, v in list(r["per_kernel"].items())[:14]:
        print(f"   {k:40s} {v['launches']/d['steps']:5.1f}/step {v['avg_us']:8.1f}us {v['share_s']*1e3/d['steps']:7.2f}ms/step")
PY
