#!/bin/bash
# round 4: RCCL on the box (world-1 collectives test), then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_rccl.log 2>&1; rc=$?
echo "rccl rc=$rc"; grep -E "RCCL|passed|failed|Error" gpurun_out/r4_rccl.log | tail -5; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/r4_bench.err; exit $rc
