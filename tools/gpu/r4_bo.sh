#!/bin/bash
# (measured neutral: BO_UN was removed again; re-add it to rerun)
# round 4: block_out with four rows per trip (production) against two
# (diagnostic build art-sbir_amd/build_var/libbo2.so, elementwise.hip with
# -DBO_UN=2): C2 legs alternated, then the block-output parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in bo2 bo4 bo2 bo4; do
  if [ $v = bo4 ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/lib$v.so; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess > gpurun_out/r4_bo_$v.json 2> gpurun_out/r4_bo_$v.err || { tail -20 gpurun_out/r4_bo_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline']['per_kernel'];print('$v C2',d['value'],d['ms_per_step'],{k:round(v['avg_us'],1) for k,v in r.items() if 'block_out' in k})" gpurun_out/r4_bo_$v.json
done
unset ARTSBIR_LIB
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_modules_gpu.py tests/test_c2_gpu.py -m gpu > gpurun_out/r4_bo_tests.log 2>&1 || { tail -30 gpurun_out/r4_bo_tests.log; exit 1; }
tail -1 gpurun_out/r4_bo_tests.log
