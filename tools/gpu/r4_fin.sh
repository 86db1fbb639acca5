#!/bin/bash
# round 4: LDS-free BatchNorm finalizes: their parity tests and the C2 / C1 /
# encoder GPU tests, the C2 bench leg, and a rocprofv3 kernel trace of it for
# tools/step_timeline.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_finalize_gpu.py tests/test_c2_gpu.py tests/test_c1_gpu.py tests/test_encoder_gpu.py tests/test_modules_gpu.py -m gpu > gpurun_out/r4_fin_tests.log 2>&1 || { tail -30 gpurun_out/r4_fin_tests.log; exit 1; }
tail -2 gpurun_out/r4_fin_tests.log
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_fin_bench$i.json 2> gpurun_out/r4_fin_bench$i.err || { tail -20 gpurun_out/r4_fin_bench$i.err; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('C2',d['value'],d['ms_per_step'])" gpurun_out/r4_fin_bench$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_fin -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-profile > $R/gpurun_out/r4_fin_prof.json 2> $R/gpurun_out/r4_fin_prof.err || { tail -20 $R/gpurun_out/r4_fin_prof.err; exit 1; }
echo prof done
