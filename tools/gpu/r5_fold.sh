#!/bin/bash
# round 5: the BatchNorm backward folded through the 1x1 convs (csrc/fold.hip):
# its kernel tests, the C2 / C1 / batched-branch parity tests with the fold on
# (the default), then the C2 step with and without it on the same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_fold_gpu.py > gpurun_out/r5_fold_tests.log 2>&1; rc=$?
echo "fold tests rc=$rc"; tail -15 gpurun_out/r5_fold_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 900 $T tests/test_c2_gpu.py tests/test_c1_gpu.py tests/test_fused_gpu.py::test_forward_branches_matches_separate_calls tests/test_modules_gpu.py tests/test_encoder_gpu.py > gpurun_out/r5_c2_tests.log 2>&1; rc=$?
echo "c2 tests rc=$rc"; tail -15 gpurun_out/r5_c2_tests.log; [ $rc = 0 ] || exit 1
B="python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 10 --warmup 3"
timeout -k 10 400 $B > gpurun_out/r5_fold_on.json 2> gpurun_out/r5_fold_on.err || { echo BENCH_ON_FAILED; tail -20 gpurun_out/r5_fold_on.err; exit 1; }
ARTSBIR_FOLD_BN=0 timeout -k 10 400 $B > gpurun_out/r5_fold_off.json 2> gpurun_out/r5_fold_off.err || { echo BENCH_OFF_FAILED; tail -20 gpurun_out/r5_fold_off.err; exit 1; }
python - <<'EOF'
import json
for n in ("on", "off"):
    d = json.loads(open(f"gpurun_out/r5_fold_{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d.get("loss_step0_rel_diff"))
EOF
