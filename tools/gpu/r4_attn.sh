#!/bin/bash
# fused attention backward vs the two-kernel form at the C5 shape (timing and
# bitwise equality of dqkv), then the attention / C5 tests
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
O=gpurun_out/r4_attn.txt
timeout -k 10 120 python3 tools/attn_bench.py --dump gpurun_out/dq_fused.pt > $O 2>&1 &&
ARTSBIR_ATTN_FWD0=1 ARTSBIR_ATTN_BWD2=1 timeout -k 10 120 python3 tools/attn_bench.py --dump gpurun_out/dq_two.pt >> $O 2>&1 &&
timeout -k 10 120 python3 tools/attn_bench.py >> $O 2>&1 &&
python3 tools/attn_bench.py --compare gpurun_out/dq_fused.pt gpurun_out/dq_two.pt >> $O 2>&1 &&
rm -f gpurun_out/dq_*.pt &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_block.py tests/test_c5_gpu.py -m gpu > gpurun_out/r4_attn_tests.log 2>&1
rc=$?; cat $O; tail -3 gpurun_out/r4_attn_tests.log; exit $rc
