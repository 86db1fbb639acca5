#!/bin/bash
# round 6: the fold-parity, tune-table and fallback-fix tests on one MI355X.
#   r6_tests.sh A   fold kernels + the committed tune table at its shapes
#   r6_tests.sh B   C2 / C1 model parity (folded BN backward under the oracle)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, timeout, pytest args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" python -u -m pytest "$@" -v --timeout-method thread -s > "gpurun_out/r6_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "gpurun_out/r6_$name.log"
  return $rc
}
case "$1" in
  A) run fold_tests 450 tests/test_fold_gpu.py --timeout 300; r=$?
     [ $r -gt 1 ] && exit $r
     run tune_tests 600 tests/test_tune_table_gpu.py --timeout 300; r2=$?
     exit $(( r | r2 )) ;;
  B) run c2c1_tests 1100 tests/test_c2_gpu.py tests/test_c1_gpu.py --timeout 900 ;;
esac
