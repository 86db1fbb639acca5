#!/bin/bash
# round 4: loader-free halo weight gradients (candidates 38/39, table entries)
# and the register-capped 32 -> 32 halo conv: parity tests of both kernels, the
# C2 GPU tests, two C2 bench legs and a kernel trace of a third
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pgemm_gpu.py tests/test_fused_gpu.py tests/test_c2_gpu.py tests/test_c1_gpu.py -m gpu -k "wgrad or 21 or c2 or c1 or C1 or C2" > gpurun_out/r4_wg2_tests.log 2>&1 || { tail -30 gpurun_out/r4_wg2_tests.log; exit 1; }
tail -1 gpurun_out/r4_wg2_tests.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_wg2_bench$i.json 2> gpurun_out/r4_wg2_bench$i.err || { tail -20 gpurun_out/r4_wg2_bench$i.err; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('C2',d['value'],d['ms_per_step'])" gpurun_out/r4_wg2_bench$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wg2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-profile > $R/gpurun_out/r4_wg2_prof.json 2> $R/gpurun_out/r4_wg2_prof.err || { tail -20 $R/gpurun_out/r4_wg2_prof.err; exit 1; }
echo prof done
