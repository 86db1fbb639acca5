#!/bin/bash
# round 6: bn1 folded through conv1 (the y-side fold) — unit tests, the engine
# toggle and the existing fold tests; then (B) the C1 / C2 model parity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" python -u -m pytest "$@" -v --timeout-method thread -s > "gpurun_out/r6_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "gpurun_out/r6_$name.log"
  return $rc
}
case "$1" in
  A) run fold_y_tests 500 -x tests/test_fold_y_gpu.py tests/test_fold_gpu.py --timeout 300 ;;
  B) run c2c1_fold1_tests 1100 tests/test_c2_gpu.py tests/test_c1_gpu.py --timeout 900 ;;
esac
