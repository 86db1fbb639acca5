#!/bin/bash
# round 5: forward-conv epilogue store variants (PG_FWD_ST builds in
# art-sbir_amd/build_var: 1 non-temporal, 2 pixel tiles outside the channel
# pairs, 3 both) on the persistent 1x1 forward (candidates 10 / 15), and the
# triplet-loss kernel tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_losses_gpu.py > gpurun_out/r5_loss_tests.log 2>&1; rc=$?
echo "loss tests rc=$rc"; tail -2 gpurun_out/r5_loss_tests.log; [ $rc = 0 ] || exit 1
for v in base 1 2 3; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libst$v.so; fi
  echo "== $v"
  ONLY=0,1,2,3,4 CFGS=10,15 timeout -k 10 300 python3 -u tools/fwd_bench.py 2>&1 | grep "stats1" || exit 1
done
