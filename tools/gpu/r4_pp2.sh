#!/bin/bash
# round 4: pp256 stamps + NT/conv A/B (one box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python -u tools/pp_stamp.py 302592 768 2304 > gpurun_out/r4_stamp.log 2>&1; rc=$?
grep -A16 "^22" gpurun_out/r4_stamp.log; [ $rc = 0 ] || exit 1
timeout -k 10 500 python -u tools/pp_bench.py --cands ${CANDS:-0,22,23} --rounds 2 ${PPARGS} > gpurun_out/r4_pp_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -v "round" gpurun_out/r4_pp_bench.log; exit $rc
